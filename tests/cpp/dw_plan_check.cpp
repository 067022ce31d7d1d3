// Host-only check of the weight-gradient work plan (lcn_internal.h DwPlan,
// make_dw_plan, make_dw_wgmap): for every batch size and group count tried,
// each (group, item) is covered by exactly one workgroup, each (group, partial
// slot) is written by exactly one workgroup, and the XCD lists are balanced.
// Built and run by tests/test_dw_plan.py (hipcc --cuda-host-only).
#include <cstdio>
#include <map>
#include <vector>

#include "lcn_internal.h"

using namespace lcn;

int main() {
  const long Bs[] = {1, 31, 64, 65, 200, 512, 1000, 2048, 2560, 2570, 4096, 8192, 16384, 30000, 32768, 65536, 131072};
  const int Gs[] = {9, 17, 93, 128, 129, 2312};
  int checked = 0;
  for (long B : Bs)
    for (int G : Gs)
      for (int slots : {1024, 768, 0}) {
        const DwPlan p = make_dw_plan(B, G, slots, 32, 128);
        const std::vector<int4> map = make_dw_wgmap(G, p, B);
        const int n_items = (int)((B + p.item_rows - 1) / p.item_rows);
        if (p.item_rows % 32 || p.n_slots < 1 || p.n_slots > 128 || map.size() % 8) {
          std::printf("bad plan B=%ld G=%d: item_rows %d n_slots %d map %zu\n", B, G, p.item_rows, p.n_slots, map.size());
          return 1;
        }
        std::vector<int> cover((size_t)G * n_items, 0), slot((size_t)G * p.n_slots, 0), per_xcd(8, 0);
        for (size_t b = 0; b < map.size(); ++b) {
          const int4 e = map[b];
          if (e.x < 0) continue;
          if (e.x >= G || e.y < 0 || e.y >= p.n_slots) { std::printf("entry out of range\n"); return 1; }
          slot[(size_t)e.x * p.n_slots + e.y]++;
          per_xcd[b & 7]++;
          for (int i = 0; i < e.w; ++i) {
            const long it = e.z + (long)i * p.stride;
            if (it * p.item_rows >= B) break;  // the kernel stops at the end of the batch
            if (it >= n_items) { std::printf("item out of range\n"); return 1; }
            cover[(size_t)e.x * n_items + it]++;
          }
        }
        for (int v : cover) if (v != 1) { std::printf("B=%ld G=%d slots=%d: an item covered %d times\n", B, G, slots, v); return 1; }
        for (int v : slot) if (v != 1) { std::printf("B=%ld G=%d slots=%d: a partial slot written %d times\n", B, G, slots, v); return 1; }
        if (p.stride == 8)
          for (int x = 1; x < 8; ++x)
            if (per_xcd[x] != per_xcd[0]) { std::printf("B=%ld G=%d: XCD lists differ\n", B, G); return 1; }
        ++checked;
      }
  std::printf("OK %d plans\n", checked);
  return 0;
}
