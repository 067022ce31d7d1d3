// Host-only check of the output-slab pairing of the forward / backward-data
// GEMM (lcn_internal.h PairPlan, make_pair_plan): every output slab is in
// exactly one pair, every (output slab, block) of the CSR lists appears in
// exactly one merged entry of its pair with its own input slab, the merged
// lists ascend, and the pairing saves what the best matching saves on the
// 17-joint skeleton (72 of 175 loads at knn 3).
// Built and run by tests/test_dw_plan.py (hipcc --cuda-host-only).
#include <cstdio>
#include <set>
#include <vector>

#include "lcn_internal.h"

using namespace lcn;

static const int kNbr[17][7] = {{1, 4, 7, -1}, {0, 7, 2, -1}, {1, 3, -1}, {2, -1}, {0, 7, 5, -1},
                                {4, 6, -1}, {5, -1}, {1, 0, 4, 14, 8, 11, -1}, {7, 9, 11, 14, -1},
                                {8, 10, -1}, {9, -1}, {8, 7, 12, -1}, {11, 13, -1}, {12, -1},
                                {8, 7, 15, -1}, {14, 16, -1}, {15, -1}};

static int check(int knn, int spj, int expect_saved) {
  const int J = 17, S = J * spj;
  std::vector<int> A(J * J, 0);
  for (int i = 0; i < J; ++i) {
    A[i * J + i] = 1;
    for (int k = 0; kNbr[i][k] >= 0; ++k) A[i * J + kNbr[i][k]] = 1;
  }
  std::vector<int> N = A;
  for (int p = 1; p < knn; ++p) {
    std::vector<int> T(J * J, 0);
    for (int i = 0; i < J; ++i)
      for (int j = 0; j < J; ++j)
        for (int k = 0; k < J; ++k) T[i * J + j] |= N[i * J + k] && A[k * J + j];
    N = T;
  }
  if (knn == 0) N.assign(J * J, 1);  // the exponential mask: every joint pair
  std::vector<int> ptr(1, 0);
  std::vector<int2> idx;
  int nblk = 0;
  std::vector<int> bid(S * S, -1);
  for (int si = 0; si < S; ++si)
    for (int so = 0; so < S; ++so)
      if (N[(si / spj) * J + so / spj]) bid[si * S + so] = nblk++;
  for (int so = 0; so < S; ++so) {
    for (int si = 0; si < S; ++si)
      if (bid[si * S + so] >= 0) idx.push_back(make_int2(si, bid[si * S + so]));
    ptr.push_back((int)idx.size());
  }
  const PairPlan p = make_pair_plan(ptr, idx, S);
  std::vector<int> seen_slab(S, 0);
  std::set<int> seen_blk;
  int saved = 0;
  for (const int4& q : p.pairs) {
    if (q.x < 0 || q.x >= S || q.y >= S || q.y == q.x || q.z >= q.w) { std::printf("bad pair\n"); return 1; }
    seen_slab[q.x]++;
    if (q.y >= 0) seen_slab[q.y]++;
    int last = -1;
    for (int e = q.z; e < q.w; ++e) {
      const int4 m = p.ment[e];
      if (m.x <= last || (m.y < 0 && m.z < 0) || (q.y < 0 && m.z >= 0)) { std::printf("bad entry\n"); return 1; }
      last = m.x;
      if (m.y >= 0) { if (bid[m.x * S + q.x] != m.y || !seen_blk.insert(m.y).second) { std::printf("bad block A\n"); return 1; } }
      if (m.z >= 0) { if (bid[m.x * S + q.y] != m.z || !seen_blk.insert(m.z).second) { std::printf("bad block B\n"); return 1; } }
      if (m.y >= 0 && m.z >= 0) ++saved;
    }
  }
  for (int s = 0; s < S; ++s) if (seen_slab[s] != 1) { std::printf("slab %d in %d pairs\n", s, seen_slab[s]); return 1; }
  if ((int)seen_blk.size() != nblk || saved != p.saved) { std::printf("blocks %zu of %d, saved %d vs %d\n", seen_blk.size(), nblk, saved, p.saved); return 1; }
  if (expect_saved >= 0 && saved != expect_saved) { std::printf("knn %d spj %d: saved %d, expected %d\n", knn, spj, saved, expect_saved); return 1; }
  std::vector<char> ord(p.pairs.size(), 0);
  for (int o : p.order) { if (o < 0 || o >= (int)ord.size() || ord[o]) { std::printf("bad order\n"); return 1; } ord[o] = 1; }
  if (p.order.size() != p.pairs.size()) { std::printf("order size\n"); return 1; }
  return 0;
}

int main() {
  // expected savings: the exact matching on the skeleton (one slab per joint)
  if (check(1, 1, 19) || check(2, 1, 43) || check(3, 1, 72) || check(4, 1, 107) || check(5, 1, 128)) return 1;
  // several slabs per joint: the slabs of a joint pair up (whole lists shared)
  if (check(3, 2, 175 * 2) || check(3, 4, 175 * 4 * 2) || check(0, 4, 289 * 4 * 2) || check(3, 3, -1) || check(0, 1, -1)) return 1;
  std::printf("OK\n");
  return 0;
}
