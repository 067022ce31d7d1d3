// Internal declarations shared by the kernel translation units and the C-ABI
// host code (lcn_api.cpp).  gfx950 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

namespace lcn {

constexpr int kJ = 17;          // joints (models_att.py:512-513)
constexpr int kSlab = 64;       // feature slab = MFMA tile edge; F is a multiple of it
constexpr int kRT = 32;         // rows per row tile of the activation layout
#ifdef EXP_GEMM_WAVES8  // diagnostic build: 8 row tiles per workgroup (half the weight LDS-DMA per wave)
constexpr int kGemmWaves = 8;
#else
constexpr int kGemmWaves = 4;   // row tiles (one per wave) per block-sparse GEMM workgroup
#endif
constexpr int kGemmRows = kRT * kGemmWaves;  // rows per workgroup = per BN partial

// ----------------------------------------------------------------------------
// Activation layout ("row tiles").  Every activation the step keeps in HBM --
// x, z, h, g, dh, dg, dz, y, dy -- with C = S*64 columns is stored as
//   [ceil(B/32)][S][8][64][4] floats:
// row tile rt (32 rows) x slab sl (64 features) is one contiguous 8 KB block;
// its 1 KB chunk g holds, for lane l = 0..63, row 32*rt + (l & 31) and the four
// features 64*sl + 8*g + 4*(l >> 5) + 0..3.  That chunk is exactly one wave's
// operand fragment of v_mfma_f32_32x32x2_f32 with the batch on the MFMA's j
// side (lane l supplies B[k = 8g + 4(l>>5) + s][j = l & 31] at k-step s), and
// exactly a wave's accumulator when the output features are on the i side
// (lane l holds D[i = 8q + 4(l>>5) + s][j = l & 31] in acc[4q + s]): every
// GEMM operand load and result store is one coalesced 1 KB transaction and
// the output of one layer is the next layer's operand without re-layout.
// Rows past B in the last tile are padding: computed, never counted.
// ----------------------------------------------------------------------------
__host__ __device__ inline int64_t tix(int64_t b, int c, int S) {
  const int sl = c >> 6, f = c & 63;
  return ((((b >> 5) * S + sl) * 8 + (f >> 3)) * 64 + (b & 31) + 32 * ((f >> 2) & 1)) * 4 + (f & 3);
}
__host__ __device__ inline int64_t tiled_floats(int64_t B, int S) { return ((B + 31) / 32) * 32 * 64 * (int64_t)S; }

// Fragment-packed 64x64 weight block ("[n][k]" with k the reduction index):
//   [g = k>>3][half = n>>5][lane = (n & 31) + 32*((k>>2)&1)][s = k & 3]
// chunk (g, half) is the MFMA i-side operand of k-group g for outputs
// 32*half..32*half+31 -- again one contiguous 1 KB read per wave.
__host__ __device__ inline int frag_ix(int n, int k) {
  return (((k >> 3) * 2 + (n >> 5)) * 64 + (n & 31) + 32 * ((k >> 2) & 1)) * 4 + (k & 3);
}

// ----------------------------------------------------------------------------
// Dropout, tf.nn.dropout(y, rate) after every BN + LeakyReLU of the training
// graph (models_att.py:673, 700, 742).  The mask is counter based, so the
// backward regenerates it instead of storing it: element (row b, column c) of
// BN layer k in one training step is kept iff
//   ((fmix32(fmix32(lo ^ lseed) + hi) >> 8) * 2^-24) >= rate,
// key = (row0 + b) * H + c = hi:lo, lseed = fmix32(step_seed ^ (k+1)*0x9e3779b9)
// (set by the host per step and layer); a kept value is x * scale with
// scale = float(1 / (1 - rate)), as TF's dropout computes it, a dropped one 0.
// oracle/lcn_oracle.py restates the same function (dropout_mask).
// ----------------------------------------------------------------------------
// Rows of the running step over all data-parallel ranks.  With several ranks
// the shards may differ in size, so the global row count (BN statistics, loss
// scale) and this rank's first global row (dropout keys) are exchanged on the
// device at the start of every step and read from here by the kernels.
struct RowInfo {
  double rows_global;   // sum of the ranks' batch rows
  int64_t row0;         // rows of the ranks below this one
};

struct Dropout {
  uint32_t lseed;   // per step and BN layer
  float rate;       // 0 = off
  float scale;
  int H;            // columns of the layer (17 * F)
  int64_t row0;     // global row of local row 0 (rank offset) when ri is null
  const RowInfo* ri;  // several ranks: row0 is read from device memory
};
// the kernel-side copy with row0 resolved (one scalar load per kernel)
__device__ inline Dropout drop_resolve(Dropout d) {
  if (d.ri) d.row0 = d.ri->row0;
  return d;
}
__host__ __device__ inline uint32_t fmix32(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
  return x;
}
__host__ __device__ inline bool drop_keep(const Dropout& d, int64_t row, int col) {
  const uint64_t key = (uint64_t)(d.row0 + row) * (uint64_t)d.H + (uint64_t)col;
  const uint32_t x = fmix32(fmix32((uint32_t)key ^ d.lseed) + (uint32_t)(key >> 32));
  return (float)(x >> 8) * 5.9604644775390625e-8f >= d.rate;
}
// x * scale if kept, else 0
__host__ __device__ inline float drop_apply(const Dropout& d, int64_t row, int col, float x) {
  return drop_keep(d, row, col) ? x * d.scale : 0.f;
}

// ----------------------------------------------------------------------------
// Block-sparse GEMM (forward z = a.We + b and backward dA = dZ.We^T).
// Output slab `so` of a row tile accumulates X[:, si-slab] . blocks[blk] over
// the (si, blk) list ptr[so]..ptr[so+1].
// ----------------------------------------------------------------------------
// operand transform applied while staging: raw, BN apply + LeakyReLU, or (the
// weight-gradient kernel's D operand) the BN + LeakyReLU backward dz from dh, z
enum { PRO_RAW = 0, PRO_BNACT = 1, PRO_BNBACK = 2 };
// epilogue partials per 128-row group: EPI_BNFWD = BN statistics of the output
// (sum, M2 about the tile mean); EPI_BNBACK = BN-backward sums of the layer
// below (sum du, sum du*zhat)
enum { EPI_NONE = 0, EPI_BNFWD = 1, EPI_BNBACK = 2 };

struct GemmArgs {
  const float* X; int S_in;          // operand activations (tiled, S_in slabs)
  const float* blocks;               // fragment-packed blocks
  const int* ptr;                    // [n_out_slabs + 1]
  const int2* idx;                   // (in_slab, block id)
  const int* order;                  // output slabs by falling list length (tail schedule), or null
  int tail;                          // row-tile groups per XCD scheduled longest-list-first at the end
  int k_groups;                      // 8-feature groups of an input slab that are non-zero (5 / 7: the lift), 0 = all 8
  int n_blocks;                      // 64x64 blocks in `blocks` (bounds of the weight loads)
  const float* bias;                 // [n_out_slabs*64] or null
  int pro_mode;                      // PRO_RAW or PRO_BNACT
  const float* pro_scale;            // forward BN scale / shift of the input's layer [F]
  const float* pro_shift;
  int pro_F;                         // channels of pro_scale / pro_shift
  int spj_in;                        // input slabs per joint (channel = (si % spj)*64 + k)
  float alpha;                       // LeakyReLU slope
  float* Y; int S_out;               // output (tiled, S_out slabs)
  const float* addsrc;               // Y = acc (+ addsrc), tiled like Y; may alias Y
  int epi_mode;
  float2* stat;                      // partials [ceil(n_rt / 4)][S_out*64]
  const float* epi_z;                // EPI_BNBACK: z of the layer below (tiled like Y)
  const float* epi_scale; const float* epi_shift; const float* epi_mean; const float* epi_rstd;
  int epi_F;                         // channels of the epi_* vectors (spj of Y = epi_F/64)
  Dropout epi_drop;                  // EPI_BNBACK: dropout of the layer below (rate 0 = off)
  int B; int n_out_slabs; int n_rt;  // n_rt = ceil(B / 32)
  // two output slabs per workgroup (gemm_pair.hip; PairPlan below), or null
  const int4* pairs;                 // [n_pairs]: (slab A, slab B or -1, first merged entry, end)
  const int4* ment;                  // merged entries: (input slab, block of A or -1, block of B or -1, 0)
  const int* pair_order;             // pairs by falling step count (tail schedule), or null
  int n_pairs;
};
void launch_gemm_bs(const GemmArgs& a, hipStream_t s);
// the hidden layers with a.pairs set: one workgroup per (row-tile group, pair of output slabs)
void launch_gemm_bs_pair(const GemmArgs& a, hipStream_t s);
// the same for launches of few row tiles (gemm_small.hip): one row tile per
// workgroup, the slab list split over its waves; stat gets one partial per
// 32-row tile (not per 128-row group); no dropout epilogue
void launch_gemm_bs_small(const GemmArgs& a, hipStream_t s);

// Pairs of output slabs for gemm_bs_pair_kernel.  A workgroup walks the union
// of its two slabs' input lists and loads an input slab both lists hold once,
// so the slabs are paired for the largest total overlap: slabs with identical
// lists first (the slabs of one joint when a joint has several), then an exact
// maximum-weight matching of the rest (bitmask DP, up to 20 slabs; greedy
// beyond), a slab that finds no partner runs alone (slab B = -1).
//   ptr / idx: the CSR lists of launch_gemm_bs (output slab -> (input slab, block)),
//   input slabs ascending within a list.
struct PairPlan {
  std::vector<int4> pairs;   // (slab A, slab B or -1, first merged entry, end)
  std::vector<int4> ment;    // (input slab, block of A or -1, block of B or -1, 0), input slabs ascending
  std::vector<int> order;    // pair indices by falling number of block steps
  int saved = 0;             // activation loads saved per row tile (sum of the pairs' overlaps)
};
inline PairPlan make_pair_plan(const std::vector<int>& ptr, const std::vector<int2>& idx, int nslab) {
  auto list_of = [&](int so) {
    std::vector<int> l;
    for (int e = ptr[so]; e < ptr[so + 1]; ++e) l.push_back(idx[e].x);
    return l;
  };
  std::vector<std::vector<int>> L(nslab);
  for (int s = 0; s < nslab; ++s) L[s] = list_of(s);
  auto overlap = [&](int x, int y) {
    int n = 0;
    size_t i = 0, j = 0;
    while (i < L[x].size() && j < L[y].size()) {
      if (L[x][i] == L[y][j]) { ++n; ++i; ++j; }
      else if (L[x][i] < L[y][j]) ++i;
      else ++j;
    }
    return n;
  };
  std::vector<std::pair<int, int>> pr;
  std::vector<int> rest;
  std::vector<char> used(nslab, 0);
  for (int s = 0; s < nslab; ++s) {  // identical lists pair up
    if (used[s]) continue;
    int mate = -1;
    for (int u = s + 1; u < nslab && mate < 0; ++u)
      if (!used[u] && L[u] == L[s]) mate = u;
    if (mate >= 0) { used[s] = used[mate] = 1; pr.push_back({s, mate}); }
  }
  for (int s = 0; s < nslab; ++s) if (!used[s]) rest.push_back(s);
  const int n = (int)rest.size();
  if (n <= 20) {  // exact: best[mask] = largest total overlap of the slabs in mask
    std::vector<int> best((size_t)1 << n, 0), choice((size_t)1 << n, -1);
    for (unsigned mask = 1; mask < (1u << n); ++mask) {
      const int i = __builtin_ctz(mask);
      const unsigned r = mask & ~(1u << i);
      best[mask] = best[r];  // slab i alone
      choice[mask] = -1;
      for (unsigned m = r; m; m &= m - 1) {
        const int j = __builtin_ctz(m);
        const int v = best[r & ~(1u << j)] + overlap(rest[i], rest[j]);
        if (v > best[mask]) { best[mask] = v; choice[mask] = j; }
      }
    }
    for (unsigned mask = n ? (1u << n) - 1 : 0; mask;) {
      const int i = __builtin_ctz(mask), j = choice[mask];
      pr.push_back({rest[i], j >= 0 ? rest[j] : -1});
      mask &= ~(1u << i);
      if (j >= 0) mask &= ~(1u << j);
    }
  } else {
    std::vector<char> done(n, 0);
    for (;;) {
      int bi = -1, bj = -1, bv = 0;
      for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j)
          if (!done[i] && !done[j] && overlap(rest[i], rest[j]) > bv) { bv = overlap(rest[i], rest[j]); bi = i; bj = j; }
      if (bi < 0) break;
      done[bi] = done[bj] = 1;
      pr.push_back({rest[bi], rest[bj]});
    }
    for (int i = 0; i < n; ++i) if (!done[i]) pr.push_back({rest[i], -1});
  }
  std::sort(pr.begin(), pr.end());
  PairPlan p;
  std::vector<int> steps;
  for (const auto& q : pr) {
    const int A = q.first, B = q.second;
    const int beg = (int)p.ment.size();
    int ea = ptr[A], eb = B >= 0 ? ptr[B] : 0;
    const int enda = ptr[A + 1], endb = B >= 0 ? ptr[B + 1] : 0;
    while (ea < enda || eb < endb) {
      const int sa = ea < enda ? idx[ea].x : INT32_MAX, sb = eb < endb ? idx[eb].x : INT32_MAX;
      const int si = sa < sb ? sa : sb;
      int4 m = make_int4(si, -1, -1, 0);
      if (sa == si) m.y = idx[ea++].y;
      if (sb == si) m.z = idx[eb++].y;
      if (m.y >= 0 && m.z >= 0) ++p.saved;
      p.ment.push_back(m);
    }
    p.pairs.push_back(make_int4(A, B, beg, (int)p.ment.size()));
    steps.push_back((enda - ptr[A]) + (endb - (B >= 0 ? ptr[B] : 0)));
  }
  p.order.resize(p.pairs.size());
  for (size_t i = 0; i < p.order.size(); ++i) p.order[i] = (int)i;
  std::stable_sort(p.order.begin(), p.order.end(), [&](int x, int y) { return steps[x] > steps[y]; });
  return p;
}

// How a weight-gradient launch splits the batch (kernels_gemm.hip).  The batch
// is cut into items of item_rows rows (a multiple of 32).  A workgroup is
// (group of blocks, partial slot, first item, item count): it walks its items
// first, first + stride, ... and keeps its accumulators over all of them, then
// writes one partial slab per block into its slot; a block has n_slots
// partials (every slot of every group is written, so dw_reduce sums them all).
//  * few groups (cfg3: 93; make_dw_plan picks stride 8): item i belongs to XCD
//    i % 8 -- every workgroup of XCD x (workgroups b, b + 8, ... share an XCD
//    and its L2) walks items = x (mod 8), so the groups that read the same rows
//    at the same time share them through that L2.  An XCD's items are dealt in
//    rounds of falling size (1/2, 1/4, 1/8, 1/8 of them): one workgroup per
//    group and round, dispatched round by round, so the launch ends with short
//    workgroups.  With 32 equal contiguous chunks a launch was ~3 rounds of
//    ~170 us workgroups and its last 15 % ran at ~35 % residency.  Very few
//    groups (the thin layers: 9 / 17): a round's items of an XCD are further
//    cut into `sub` parts so the launch still has ~3 x the resident workgroups.
//  * many groups (the cfg4 shape: 2 312; stride 1): n_slots contiguous chunks
//    per group, one item each (item_rows = rows per chunk), tens of rounds.
struct DwPlan { int item_rows, stride, n_slots, sub; };
inline int dw_plan_slots(const DwPlan& p) { return p.n_slots; }
constexpr int kDwRounds = 4;
// groups: number of block groups; slots: workgroups the GPU holds at once;
// chunks: the contiguous-chunk count of the many-groups case; max_slots: cap on
// the partials per block
inline DwPlan make_dw_plan(int64_t B, int groups, int slots, int chunks, int max_slots) {
  DwPlan p{};
  const int64_t n64 = (B + 63) / 64;
  if (groups * 8 <= slots && 8 * kDwRounds <= max_slots && n64 >= 16) {  // (a tiny batch: plain chunks)
    // >= 64 items per XCD where the batch allows (16 for the shortest round), at most 256 rows an item
    const int64_t r = B / (8 * 64);
    p.item_rows = (int)std::min<int64_t>(256, std::max<int64_t>(64, r / 64 * 64));
    p.stride = 8;
    const int64_t per_xcd = ((B + p.item_rows - 1) / p.item_rows + 7) / 8;
    const int rounds = (int)std::max<int64_t>(1, std::min<int64_t>(kDwRounds, per_xcd / 4));
    // ~3 x the resident workgroups in all, within the partial cap and >= 2 items a workgroup
    int sub = std::max(1, (3 * slots - 96 + groups * 8 * rounds - 1) / (groups * 8 * rounds));
    sub = (int)std::min<int64_t>({(int64_t)sub, (int64_t)max_slots / (8 * rounds), std::max<int64_t>(1, per_xcd / (2 * rounds))});
    p.sub = std::max(1, sub);
    p.n_slots = 8 * rounds * p.sub;
    return p;
  }
  const int nch = (int)std::max<int64_t>(1, std::min<int64_t>(std::min(chunks, max_slots), n64));
  p.item_rows = (int)(((B + nch - 1) / nch + 63) / 64 * 64);
  p.stride = 1;
  p.sub = 1;
  p.n_slots = (int)((B + p.item_rows - 1) / p.item_rows);
  return p;
}
// The workgroups of a launch: entry b is workgroup blockIdx.x = b as (group,
// slot, first item, item count); (-1, 0, 0, 0) pads the XCD lists to equal
// length.  Stride 8: entry 8 i + x is the i-th workgroup of XCD x, rounds in
// order, groups in order within a round; a round's share of the n items of the
// XCD: n/2, n/4, ..., the last round takes the rest.
inline std::vector<int4> make_dw_wgmap(int groups, const DwPlan& p, int64_t B) {
  const int n_items = (int)((B + p.item_rows - 1) / p.item_rows);
  if (p.stride == 1) {
    std::vector<int4> map;
    for (int c = 0; c < p.n_slots; ++c)
      for (int g = 0; g < groups; ++g) map.push_back(make_int4(g, c, c, c < n_items ? 1 : 0));
    // chunk-major: the groups of a chunk are adjacent; give each XCD whole chunks
    // (a contiguous range of entries) by interleaving the ranges
    const int n = (int)map.size(), q = n >> 3, r = n & 7;
    std::vector<int4> out(8 * ((n + 7) / 8), make_int4(-1, 0, 0, 0));
    for (int x = 0; x < 8; ++x) {
      const int lo = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q, cnt = q + (x < r ? 1 : 0);
      for (int i = 0; i < cnt; ++i) out[8 * i + x] = map[lo + i];
    }
    return out;
  }
  const int sub = std::max(1, p.sub), rounds = p.n_slots / (8 * sub);
  std::vector<int4> map((size_t)8 * rounds * sub * groups, make_int4(-1, 0, 0, 0));
  for (int x = 0; x < 8; ++x) {
    const int n = n_items > x ? (n_items - x + 7) / 8 : 0;  // items x, x + 8, ... of this XCD
    int a = 0;
    for (int r = 0; r < rounds; ++r) {
      const int cnt = r + 1 < rounds ? (n - a + 1) / 2 : n - a;
      for (int u = 0; u < sub; ++u) {  // the round's items in `sub` contiguous parts
        const int lo = a + (int)((int64_t)cnt * u / sub), hi = a + (int)((int64_t)cnt * (u + 1) / sub);
        for (int g = 0; g < groups; ++g)
          map[8 * (((size_t)r * sub + u) * groups + g) + x] = make_int4(g, 8 * (r * sub + u) + x, x + 8 * lo, hi - lo);
      }
      a += cnt;
    }
  }
  return map;
}
// dWe blocks: part[chunk][blk][p][q] = sum_{b in chunk} A[b, si*64+p] * D[b, so*64+q]
// Work unit = a group of up to 2 blocks with the same output slab so (they
// share the staged D operand): int4 (so, block0, block1 or -1, rank | count << 8
// of the group among the groups of so, which take turns storing dz).
struct GemmDwArgs {
  const float* A; int S_a;           // tiled
  const float* D; int S_d;           // tiled; d_bnback: D = dh and the operand is dz
  const float* pro_scale; const float* pro_shift; int spj_a; float alpha;  // A: BN apply + act
  int d_bnback; int spj_d;
  const float* d_z; const float* d_scale; const float* d_shift; const float* d_c123; int d_F;
  float* dz_out;                     // d_bnback: dz (tiled like D) or null
  Dropout d_drop;                    // d_bnback: dropout of D's layer (rate 0 = off)
  const int2* blk;                   // (si, so) per block
  int nblk;
  const int4* groups; int ngroups;   // block groups (see above)
  int B; DwPlan plan;                // how the batch is split (see DwPlan)
  const int4* wgmap; int n_wg;       // the launch's workgroups (make_dw_wgmap)
  float* part;                       // [dw_plan_slots(plan)][nblk][4096]
#ifdef EXP_CLOCK
  uint64_t* clk;                     // diagnostic build: per workgroup (shader clocks, 100 MHz ticks, start, end)
#endif
};
void launch_gemm_dw(const GemmDwArgs& a, hipStream_t s);
// workgroups of the weight-gradient kernel the current device holds at once
int gemm_dw_resident_slots();
// four blocks of an output slab per workgroup (gemm_dw4.hip): two int4 per
// group, (so, 4, rank, count) and (b0, b1, b2, b3)
void launch_gemm_dw4(const GemmDwArgs& a, hipStream_t s);
int gemm_dw4_resident_slots();
// sum partials over chunks; write into dense dW [rows][ld] at (si*64+p, so*64+q),
// dropping rows >= rows_valid / columns >= cols_valid (padding of thin layers)
void launch_dw_reduce(const float* part, int nchunks, int nblk, const int2* blk,
                      float* dW, int ld, int rows_valid, int cols_valid, hipStream_t s);

// ----------------------------------------------------------------------------
// The thin layers run on the same MFMA kernels with the narrow side padded to
// one 64-wide slab: the lift's input x [B][17*in_F] is a 1-slab tiled buffer
// (K = 34 -> 64, zero padded) and the output layer's 51 columns live in 1-slab
// tiled buffers.
// ----------------------------------------------------------------------------
// row-major src [B][cols] (cols <= 64) -> 1-slab tiled dst, zero padded (rows
// of the last tile past B and columns past cols)
void launch_tile_in(const float* src, int cols, int B, float* dst, hipStream_t s);
// y = h . W4e from the GEMM; out[b, 3j+c] = (c < 2 ? x[b, in_f*j+c] : 0) + (y + b4);
// loss partials and dy = dscale * (out - lab) (models_att.py:765-773, :356)
struct OutAsmArgs {
  const float* y;                    // 1-slab tiled (51 used)
  const float* b4;                   // [51]
  const float* x; int in_f;          // 1-slab tiled
  const float* lab;                  // [B][51] row-major, or null
  float* out;                        // [B][51] row-major
  float* dy;                         // 1-slab tiled, or null (padding written as 0)
  double* loss_part;                 // [gridDim] or null
  double* db_part;                   // [gridDim][64] column sums of dy (the output bias gradient), or null
  double rows;                       // global batch rows: dy = 2 (out - lab) / (rows * 51)
  const RowInfo* ri;                 // several ranks: rows read from device memory
  int B;
};
void launch_out_assemble(const OutAsmArgs& a, int grid, hipStream_t s);

// ----------------------------------------------------------------------------
// Device-resident datasets (kernels_data.hip): permutation gather into the
// lift operand, test-time augmentation copies and their undo + mean.
// ----------------------------------------------------------------------------
enum { kF32 = 0, kF64 = 1 };
enum { kAugNone = 0, kAugFlip = 1, kAugRotate = 2, kAugTranslate = 3 };
constexpr int kMaxCopies = 8;
// copies of the virtual dataset: op / parameters per copy (rotate: p0 = cos,
// p1 = sin of the angle; translate: p0 = t)
struct Augment {
  int n_copies;
  int op[kMaxCopies];
  double p0[kMaxCopies], p1[kMaxCopies];
};
// x rows v = idx[b] (or base + b) of the augmented dataset [rows][17*k] ->
// 1-slab row tiles of B rows (zero rows outside the virtual range / past B)
void launch_gather_x(const void* ds, int dtype, int64_t rows, int k, const int* idx, int64_t base,
                     const Augment& aug, int B, float* dst, hipStream_t s);
// rows v = idx[b] (or base + b) of ds [rows][cols] -> float32 row-major [B][cols]
void launch_gather_rows(const void* ds, int dtype, int64_t rows, int cols, const int* idx,
                        int64_t base, int B, float* dst, hipStream_t s);
void launch_store_pred(const float* out, int64_t n, double* pred, hipStream_t s);
void launch_tta_undo(const double* pred, int64_t N, const Augment& undo, double* out, hipStream_t s);
// losses[i] = (float)(loss_sum / (rows * 51)); rows from ri when given
void launch_batch_loss(const double* loss_sum, double rows, const RowInfo* ri, float* losses, int i,
                       hipStream_t s);
// rows[r] = (r == rank ? B : 0) for r < world: the all-reduce (sum) of it is the
// all-gather of the ranks' batch rows
void launch_rows_begin(double* rows, int world, int rank, int64_t B, hipStream_t s);
// rows[world] of every rank -> RowInfo of this rank
void launch_rows_finish(const double* rows, int world, int rank, RowInfo* ri, hipStream_t s);
// evaluate.py per-frame, per-joint error (kernels_eval.hip): pred / gt [n][17][3],
// box [n][4], cam [n][4] = (cx, cy, fx, fy), root_depth [n] -> err [n][17]
void launch_mpjpe(int64_t n, const double* pred, const double* gt, const double* box, const double* cam,
                  const double* root_depth, int protocol2, double* err, hipStream_t s);

// message of a failed handle-free entry point, returned by lcn_last_error(NULL)
// (per thread; lcn_api.cpp)
void set_global_error(const std::string& msg);

// ----------------------------------------------------------------------------
// BatchNorm (batch statistics), activation, BN backward
// ----------------------------------------------------------------------------
// stats per channel: mean, rstd, scale = gamma*rstd, shift = beta - mean*scale
struct BnStats { float* mean; float* rstd; float* scale; float* shift; };
// float64 column sums of tile partials part[n_tiles][H] into kColSplit
// tile-group partials out[kColSplit][H] (added up by the finish kernels):
//   mode 0 (sum x, sum y); mode 1 (sum x, sum (y + x^2 / rows_of_tile))
constexpr int kColSplit = 8;
void launch_colreduce(const float2* part, int n_tiles, int tile_rows, int B, int H, int mode,
                      double2* out, hipStream_t s);
// The GEMM epilogue's tile partials, handed to the finish kernels directly when
// a launch has few tiles (part == null: they read colreduce's sums instead).
struct TilePartials {
  const float2* part; int n_tiles, tile_rows, B;
};
// Values that ride on a SyncBN all-reduce, appended to its 2F channel sums at
// acc[2F ..], so a data-parallel step needs no collective of their own:
//   kRideRows (forward, BN layer 0): the ranks' batch rows, one slot per rank
//     (phase 1 fills this rank's slot, the all-reduce sums the one-hot vectors,
//     phase 2 derives this rank's RowInfo and uses the global row count);
//   kRideLoss (the first BN backward of a step): the rank's loss sum, one slot
//     (phase 1 reads *loss, phase 2 writes the all-reduced sum back).
enum { kRideNone = 0, kRideRows = 1, kRideLoss = 2 };
struct BnRider {
  int kind;
  int world, rank;      // kRideRows
  double b_local;       // kRideRows: this rank's batch rows
  RowInfo* ri_out;      // kRideRows: written by phase 2
  double* loss;         // kRideLoss
};
inline int rider_slots(const BnRider& r) { return r.kind == kRideRows ? r.world : r.kind == kRideLoss ? 1 : 0; }
// forward BN finish from colreduce mode-1 sums.  phase 0 complete (single GPU);
// 1 local channel sums -> acc[2F]; 2 finish from all-reduced acc.  The element
// count per channel is rows_global * J, rows_global = `rows` or, when ri is
// given, ri->rows_global.  zsum (optional): per-column sum of z.
void launch_bn_fwd_finalize(const double2* col, const TilePartials& tp, int H, int F, int phase,
                            double rows, const RowInfo* ri,
                            const float* gamma, const float* beta, float eps, double* acc,
                            BnStats st, double* zsum, const BnRider& rider, hipStream_t s);
// backward BN finish from colreduce mode-0 sums of (du, du*zhat): c1|c2|c3,
// local dgamma/dbeta and the bias gradient db; bn = 0: db = sum du only
void launch_bn_bwd_finalize(const double2* col, const TilePartials& tp, int H, int F, int phase,
                            int bn, double rows, const RowInfo* ri, double b_local, const float* gamma, const float* mean,
                            const float* rstd, double* acc, float* dgamma, float* dbeta,
                            float* c123, const double* zsum, float* db, const BnRider& rider,
                            hipStream_t s);
// colreduce and the finish (phase 0 or 1) in ONE launch: the workgroup that
// finishes its column sums last runs the finish (kernels_elem.hip).  `ticket`:
// a device int that is 0 before the launch (the kernel leaves it 0).
void launch_colreduce_bn_fwd(const float2* part, int n_tiles, int tile_rows, int B, double2* col,
                             int* ticket, int H, int F, int phase, double rows, const RowInfo* ri,
                             const float* gamma, const float* beta, float eps, double* acc, BnStats st,
                             double* zsum, const BnRider& rider, hipStream_t s);
void launch_colreduce_bn_bwd(const float2* part, int n_tiles, int tile_rows, int B, double2* col,
                             int* ticket, int H, int F, int phase, int bn, double rows,
                             const RowInfo* ri, double b_local, const float* gamma, const float* mean,
                             const float* rstd, double* acc, float* dgamma, float* dbeta, float* c123,
                             const double* zsum, float* db, const BnRider& rider, hipStream_t s);
// h = [res +] leaky(scale*z + shift), tiled [B][S*64] buffers
void launch_bn_act(const float* z, const float* res, float* h, const float* scale,
                   const float* shift, int F, float alpha, int B, int S, const Dropout& drop,
                   hipStream_t s);
// sums the n workgroup partials of out_assemble: the loss, and (db_part given)
// the 51 columns of dy into the output layer's bias gradient db_out
void launch_loss_finalize(const double* part, int n, double* out, const double* db_part, float* db_out,
                          hipStream_t s);

// ----------------------------------------------------------------------------
// Parameters: mask, clip_by_norm, masking, packing, gradients, Adam
// ----------------------------------------------------------------------------
struct WLayer {            // one linear layer's weight
  int64_t w_off;           // offset in the flat parameter vector
  int kin, nout, fin, fout;
  int kind;                // 0 lift, 1 hidden, 2 output
  // 64x64 blocks of W_e for the MFMA kernels, [n][k] fragment-packed (frag_ix):
  //   hidden: blk_fwd [nblk][q][p], blk_bwd [nblk][p][q]
  //   lift:   blk_fwd [nslab][f][k = u*in_F + c] (k >= 17*in_F zero)
  //   output: blk_fwd [nslab][c'][p], blk_bwd [nslab][p][c'] (c' >= 51 zero)
  float* blk_fwd;
  float* blk_bwd;
  const int2* blk;         // hidden: (si, so) per block (device)
  int nblk;
};
// M = softmax(V,0) (.) C  (LC)  or M = const (EXP); writes M and S
void launch_mask(const float* V, const float* Cmat, int learnable, float* M, float* S,
                 hipStream_t s);
// sum of squares per layer -> norm2[l] (double); denom[l] = max(sqrt, 1) (float)
void launch_wnorm(const float* params, const int64_t* offs, const int64_t* sizes, int nl,
                  double* part, int parts_per_layer, double* norm2, float* denom, int max_norm,
                  hipStream_t s);
// W_e = (W / denom) * M[i,j]; writes the layer's packed forms (thin layers)
void launch_wprep(const float* params, const WLayer& L, const float* M, const float* denom,
                  int layer, hipStream_t s);
// the same for all hidden layers in one launch
struct WPrepHidden {
  int64_t w_off;           // the layer's weight in the flat parameter vector
  float* fwd; float* bwd;  // its packed block arrays
  int layer;               // index into denom
};
void launch_wprep_hidden(const float* params, const WPrepHidden* items, int n_layers, int ld,
                         const int2* blk, int nblk, int spj, const float* M, const float* denom,
                         hipStream_t s);
// blocksum[l][i][j] = sum_{p,q} dWe * W over joint block (i,j)
void launch_wdot(const float* rg, const float* params, const int64_t* offs, const int* kin,
                 const int* nout, int nl, double* blocksum, hipStream_t s);
// dM, dV (LC) and per-layer clip coefficients coef[l] = (1/denom, c_l)
void launch_maskgrad(const double* blocksum, int nl, const float* M, const float* S,
                     const float* Cmat, int learnable, const float* denom, const double* norm2,
                     int max_norm, float* dV, float* lcoef, hipStream_t s);

// Segment of the flat parameter vector for the fused gradient-finish + Adam.
struct AdamSeg {
  int64_t off, size;
  int kind;                // 0 plain (bias/gamma/beta/mask), 1 weight (clip+mask backward)
  int layer;               // weight: index into lcoef
  int cols, fin, fout;     // weight geometry
  int reg;                 // add regularisation * theta
};
void launch_adam(float* theta, float* m, float* v, const float* rg, float* gout,
                 const AdamSeg* segs, const int64_t* seg_block_start, int nseg,
                 int64_t total_blocks, const float* M, const float* lcoef, float reg,
                 const float* lr_t_dev, float beta1, float beta2, float eps, int update, hipStream_t s);

}  // namespace lcn
