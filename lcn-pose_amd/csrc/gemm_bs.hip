// Block-sparse fp32 MFMA GEMM of the LCN layers, forward and backward-data
// (gfx950).
//
// Replaces the TF MatMul ops of cgcnn.two_linear (models_att.py:662, :692) and
// of the thin lift / output layers (:729, :765; their narrow side padded to one
// 64-wide slab), and the dX half of their autodiff.  W_e = clip(W) (.) M
// (models_att.py:576-586) is zero outside the blocks (i, j) with M[i,j] != 0,
// so a 64x64 feature block of a joint pair is the unit of work and absent
// blocks are skipped (175 of 289 present at knn=3).  Output slab `so` of a row
// tile accumulates X[:, si-slab] . block over the CSR list ptr[so]..ptr[so+1].
//
// Exact fp32: v_mfma_f32_32x32x2_f32 (gfx950 has no xf32; the f32-input MFMA
// is a k-ordered fmaf chain).  Roles: the weight block is the i-side operand
// (output features), the activations the j-side (batch rows), so
//   D[n][b] = sum_k We[n][k] X[b][k]
// and both operands and the accumulator are exactly 1 KB chunks of the
// row-tile layout (lcn_internal.h): lane l supplies X[32rt + (l&31)][8g +
// 4(l>>5) + s] at k-step s of group g and holds Y[32rt + (l&31)][8q + 4(l>>5)
// + s] in acc[4q + s].  The lane-half k permutation (lane half h takes k = 8g
// + 4h + s) makes each operand fragment one float4.
//
// Workgroup = 4 waves = 4 row tiles (128 rows) x one output slab.  Each wave
// loads its own activation fragments straight from HBM/L2 into registers (8
// coalesced 1 KB loads per input slab, prefetched one slab ahead in a second
// register set); the weight block, shared by the 4 waves, goes into a double
// LDS buffer by LDS-DMA, so there is one barrier per input slab.  The
// accumulators start at the bias; the residual and the BN-backward epilogue's z
// are loaded after the loop, ahead of the output stores (prefetching it at kernel
// start held 32 VGPRs through the loop and cost a wave per SIMD: 4 waves/SIMD
// at <= 128 VGPRs is 3 % faster for the dX GEMM).  Measured
// against a 128x64 LDS-staged tile with two barriers per slab: 124 vs 114
// TFLOP/s at B = 65 536, knn 3.
//
// Operand prologue (PRO):  PRO_RAW a = X;  PRO_BNACT a = leaky(scale X + shift)
// (BN apply + LeakyReLU of the input's layer, scale/shift tables in LDS).
// Epilogue: store; then per 128-row group either BN forward partials of the
// output (sum, M2 about the group mean) or BN backward partials of the layer
// below (sum du, sum du * zhat): column sums per wave through LDS, merged
// across the 4 waves.
#include <algorithm>

#include "gemm_epilogue.h"

namespace lcn {

#define STEP(W0, W1, XV)                 \
  acc0 = MFMA32((W0).x, (XV).x, acc0);   \
  acc1 = MFMA32((W1).x, (XV).x, acc1);   \
  acc0 = MFMA32((W0).y, (XV).y, acc0);   \
  acc1 = MFMA32((W1).y, (XV).y, acc1);   \
  acc0 = MFMA32((W0).z, (XV).z, acc0);   \
  acc1 = MFMA32((W1).z, (XV).z, acc1);   \
  acc0 = MFMA32((W0).w, (XV).w, acc0);   \
  acc1 = MFMA32((W1).w, (XV).w, acc1);

#define DECLX(P) float4 P##0, P##1, P##2, P##3, P##4, P##5, P##6, P##7;
// Operand loads are BUFFER loads: a scalar resource (base + size) with one
// 32-bit offset register per lane, the slab / block part of the address in
// scalar registers.  Beside a stream of MFMAs a load that takes a 64-bit address
// pair per lane costs matrix-core time (scripts/microbench/mfma_steps.hip: the
// slab loop's 12 loads per 64 MFMAs 83.7 % of the MFMA peak as global loads,
// 88.4 % as buffer loads, all L2 hits); reads past a resource return 0.
// activation fragments of input slab si (8 chunks of this wave's row tile):
// byte offset si * 8192 + chunk * 1024 (scalar) + lane * 16
#define LOADX(P, SI)                                                      \
  {                                                                       \
    const int so_ = (SI) * 8192;                                          \
    P##0 = BUFLD(xres, xlo, so_);          P##1 = BUFLD(xres, xlo + 1024, so_); \
    P##2 = BUFLD(xres, xlo + 2048, so_);   P##3 = BUFLD(xres, xlo + 3072, so_); \
    P##4 = BUFLD(xres, xlo, so_ + 4096);                                  \
    if constexpr (KG > 5) { P##5 = BUFLD(xres, xlo + 1024, so_ + 4096); P##6 = BUFLD(xres, xlo + 2048, so_ + 4096); } \
    if constexpr (KG > 7) P##7 = BUFLD(xres, xlo + 3072, so_ + 4096);     \
  }
// this thread's quarter of a weight block, global -> LDS buffer BUF by
// LDS-DMA (buffer_load_dwordx4 ... lds: no VGPRs, no ds_write; each wave
// instruction lands 1 KB lane-linear, which is the fragment-packed order)
#define GLDS(SOFF, DST) \
  __builtin_amdgcn_raw_ptr_buffer_load_lds(wres, (__attribute__((address_space(3))) void*)(DST), 16, xlo, (SOFF), 0, 0);
#define LOADW(BLK, BUF)                                                   \
  {                                                                       \
    const int bo_ = (BLK) * 16384 + wv_u * 1024;  /* this wave's 1 KB of each 4 KB quarter (8 KB half) */ \
    float4* d_ = Wl + (BUF) * 1024 + (threadIdx.x & ~63);                 \
    if constexpr (kGemmWaves == 8) {                                      \
      GLDS(bo_, d_)                                                       \
      if (KG > 7 || wv_u + 8 < 2 * KG) GLDS(bo_ + 8192, d_ + 512)         \
    } else {                                                              \
      GLDS(bo_, d_) GLDS(bo_ + 4096, d_ + 256) GLDS(bo_ + 8192, d_ + 512) \
      if constexpr (KG > 6) GLDS(bo_ + 12288, d_ + 768)                   \
    }                                                                     \
  }
// BN apply + LeakyReLU of one activation fragment (k-group G of a slab whose
// first channel is CH), scale / shift from the LDS tables
#define TSTEP(G, XV, CH)                                                  \
  {                                                                       \
    const int c_ = (CH) + 8 * (G) + 4 * h;                                \
    XV = bnact4(XV, *(const float4*)(tsc + c_), *(const float4*)(tsh + c_), al); \
  }
#define TRANSX(P, CH)                                                     \
  TSTEP(0, P##0, CH) TSTEP(1, P##1, CH) TSTEP(2, P##2, CH) TSTEP(3, P##3, CH) \
  TSTEP(4, P##4, CH) TSTEP(5, P##5, CH) TSTEP(6, P##6, CH) TSTEP(7, P##7, CH)
#define GSTEP(BUF, G, XV, CH)                                             \
  {                                                                       \
    const float4 w0_ = Wl[(BUF) * 1024 + (2 * (G)) * 64 + lane];          \
    const float4 w1_ = Wl[(BUF) * 1024 + (2 * (G) + 1) * 64 + lane];      \
    STEP(w0_, w1_, XV)                                                    \
  }
// schedule of one input slab: the LDS reads of group g+1 are issued before
// the 8 MFMAs of group g, so their latency hides under those MFMAs
#define SGB(MASK, N) __builtin_amdgcn_sched_group_barrier(MASK, N, 0);
#define SCHED_SLAB                                                          \
  SGB(0x100, DSR)                                                           \
  SGB(0x100, DSR) SGB(0x008, 8) SGB(0x100, DSR) SGB(0x008, 8)               \
  SGB(0x100, DSR) SGB(0x008, 8) SGB(0x100, DSR) SGB(0x008, 8)               \
  SGB(0x100, DSR) SGB(0x008, 8) SGB(0x100, DSR) SGB(0x008, 8)               \
  SGB(0x100, DSR) SGB(0x008, 8) SGB(0x008, 8)
// PRO_BNACT: the slab's eight fragments are transformed in one block ahead of
// its MFMAs (16 table reads in flight together, then 96 VALU operations the
// other waves of the SIMD cover); done per k-group between the MFMAs, every
// group waited for its own table reads (842 vs 805 us, gemm_bench cfg3)
#define COMPX_PRE(P, CH) if constexpr (PRO == PRO_BNACT) { TRANSX(P, CH) __builtin_amdgcn_sched_barrier(0); }
#define COMPX(BUF, P, CH)                                                 \
  COMPX_PRE(P, CH)                                                        \
  GSTEP(BUF, 0, P##0, CH) GSTEP(BUF, 1, P##1, CH) GSTEP(BUF, 2, P##2, CH) \
  GSTEP(BUF, 3, P##3, CH) GSTEP(BUF, 4, P##4, CH)                         \
  if constexpr (KG > 5) { GSTEP(BUF, 5, P##5, CH) GSTEP(BUF, 6, P##6, CH) } \
  if constexpr (KG > 7) { GSTEP(BUF, 7, P##7, CH) SCHED_SLAB }

// KG: k-groups (8 features each) of an input slab that are multiplied.  8 for
// the hidden layers; the lift's input slab holds 17 * in_F = 34 or 51 features
// and zeros (its weight rows there are zero too), so its instances stop after
// 5 or 7 groups: the thin layer is MFMA-bound at the padded width.

template <int PRO, int EPI, int KG = 8>
__global__ __launch_bounds__(64 * kGemmWaves) __attribute__((amdgpu_waves_per_eu(4))) void gemm_bs_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float4 Wl[];  // [2][1024] (+ BN tables)
#ifdef EXP_CLOCK
  // diagnostic build: shader-clock and 100 MHz real-time stamps around the
  // workgroup, written to a buffer of their own (a.stat is unused by EPI_NONE)
  const uint64_t ck0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  // Work map.  Workgroups b, b + 8, ... share an XCD (and its L2): each XCD
  // takes a contiguous range of row-tile groups and walks it group by group,
  // so the ~10 output slabs that read an input slab run close in time.  The
  // lists differ in length (5..17 slabs at knn 3) and a workgroup lives ~10 %
  // of the launch, so in natural order the launch ends in a long drain; the
  // last `tail` groups of each XCD are therefore issued longest list first
  // across those groups (order[]): what is still running at the end is short.
  const int nso = a.n_out_slabs;
  const int n_rtg = (a.n_rt + kGemmWaves - 1) / kGemmWaves;
  const int xcd = blockIdx.x & 7, li = blockIdx.x >> 3;
  // n_rtg = 8 base + extra: the first `extra` XCDs take one group more, so a
  // batch that is not a multiple of 1024 rows still loads every XCD
  const int base = n_rtg >> 3, extra = n_rtg & 7;
  const int g0 = xcd * base + min(xcd, extra), R = base + (xcd < extra ? 1 : 0);
  if (li >= R * nso) return;  // padding of the grid (uniform per workgroup)
  const int T = a.order ? min(R, a.tail) : 0;
  int rtg, so;
  if (li < (R - T) * nso) {
    rtg = li / nso;
    so = li - rtg * nso;
    rtg += g0;
  } else {
    const int j = li - (R - T) * nso, rank = j / T;
    so = a.order[rank];
    rtg = g0 + (R - T) + (j - rank * T);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  // the wave index and everything derived from it are wave-uniform: scalar registers
  const int wv_u = __builtin_amdgcn_readfirstlane(w);
  const int rt_raw = rtg * kGemmWaves + wv_u;
  const bool live = rt_raw < a.n_rt;
  // waves past the last row tile recompute it (they take part in the barriers)
  const int rt = live ? rt_raw : a.n_rt - 1;
  // the lift's lists are known without a load: output slab so <- block so of input slab 0
  constexpr bool kLift = KG < 8;
  const int beg = kLift ? 0 : a.ptr[so], end = kLift ? 1 : a.ptr[so + 1];
  const int2* __restrict__ idx = a.idx;
  // buffer resources: this wave's row tile of the activations (all its input
  // slabs; S_in = 0 is the microbenchmark's every-tile-reads-tile-0 mode), the
  // packed weight blocks
  const int rt_u = rt;
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)a.X + (size_t)rt_u * a.S_in * 8192), 0, (a.S_in ? a.S_in : a.n_out_slabs) * 8192, 0x00020000);
  const __amdgpu_buffer_rsrc_t wres =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.blocks, 0, a.n_blocks * 16384, 0x00020000);
  const int xlo = lane * 16;  // the one address register of every operand load
  const float al = a.alpha;
  const float* tsc = nullptr;
  const float* tsh = nullptr;
  const int spj = a.spj_in;
  constexpr int DSR = 2;  // weight reads per k-group

  // the first weight block and activation fragments go in flight first; the
  // bias / residual / table loads below are batched behind them, so the
  // prologue waits for memory once (not once per accumulator quarter)
  DECLX(xa)
  DECLX(xb)
  // list entries are wave-uniform: kept in scalar registers
#define UIDX(E) ({ const int2 t_ = idx[(E)]; make_int2(__builtin_amdgcn_readfirstlane(t_.x), __builtin_amdgcn_readfirstlane(t_.y)); })
  int2 ia = kLift ? make_int2(0, so) : UIDX(beg), ib = ia;
  LOADW(ia.y, 0)
  LOADX(xa, ia.x)
  // accumulators start at the bias (the MFMAs add onto it); the residual is
  // added after the loop, its loads in flight together with the epilogue's z
  // (what the residual costs the dX GEMM is its 285 MB of traffic: 781 us with
  // it, 757 us without; loading it ahead of the loop or after it measured the
  // same, 784 vs 781 us)
  float4 bq[8];
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.bias) {
#pragma unroll
    for (int q = 0; q < 8; ++q) bq[q] = *(const float4*)(a.bias + so * kSlab + 8 * q + 4 * h);
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) bq[q] = zero4;
  }
  if constexpr (PRO == PRO_BNACT) {  // BN scale / shift of the operand's layer -> LDS
    float* tb = (float*)(Wl + kTabOff);
    for (int c = threadIdx.x; c < a.pro_F; c += 64 * kGemmWaves) {
      tb[c] = a.pro_scale[c];
      tb[a.pro_F + c] = a.pro_shift[c];
    }
    tsc = tb;
    tsh = tb + a.pro_F;
  }
  // EPI_BNBACK: the per-channel BN constants of this output slab go to an LDS table
  float* ptab = (float*)(Wl + kTabOff);  // [4][64]: scale, shift, mean, rstd
  if constexpr (EPI == EPI_BNBACK || EPI == kEpiBnBackDrop) epi_fill_table(a, ptab, so);
  f32x16 acc0, acc1;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 b0 = bq[q], b1 = bq[4 + q];
    acc0[4 * q + 0] = b0.x; acc0[4 * q + 1] = b0.y; acc0[4 * q + 2] = b0.z; acc0[4 * q + 3] = b0.w;
    acc1[4 * q + 0] = b1.x; acc1[4 * q + 1] = b1.y; acc1[4 * q + 2] = b1.z; acc1[4 * q + 3] = b1.w;
  }
  __syncthreads();
  // every output slab has >= 1 input block (checked in lcn_create)
  for (int e = beg; e < end; e += 2) {
    const bool n1 = e + 1 < end;
    if (n1) {
      ib = UIDX(e + 1);
      LOADW(ib.y, 1)
      LOADX(xb, ib.x)
    }
    COMPX(0, xa, (ia.x % spj) * kSlab)
    __syncthreads();  // drains the LDS-DMA of buffer 1 (vmcnt(0)) and publishes it
    if (n1) {
      const bool n2 = e + 2 < end;
      if (n2) {
        ia = UIDX(e + 2);
        LOADW(ia.y, 0)
        LOADX(xa, ia.x)
      }
      COMPX(1, xb, (ib.x % spj) * kSlab)
      __syncthreads();
    }
  }

  // ---- epilogue ----
  gemm_epilogue<EPI>(a, Wl, ptab, ptab + 256, rtg, rt, live, so, acc0, acc1);
#ifdef EXP_CLOCK
  if constexpr (EPI == EPI_NONE) {
    if (threadIdx.x == 0 && a.stat) {
      const uint64_t ck1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
      ((uint64_t*)a.stat)[4 * blockIdx.x] = ck1 - ck0;
      ((uint64_t*)a.stat)[4 * blockIdx.x + 1] = rt1 - rt0;
      ((uint64_t*)a.stat)[4 * blockIdx.x + 2] = rt0;
      ((uint64_t*)a.stat)[4 * blockIdx.x + 3] = rt1;
    }
  }
#endif
}

void launch_gemm_bs(const GemmArgs& a, hipStream_t s) {
  const int n_rtg = (a.n_rt + kGemmWaves - 1) / kGemmWaves;
  const int grid = 8 * ((n_rtg + 7) / 8) * a.n_out_slabs;  // 8 XCDs x row-tile groups per XCD x slabs
  // weight double buffer; BN tables / epilogue constants and the 4-wave merge after it
  const size_t lds = 2 * 1024 * sizeof(float4);
  const size_t tab = kTabOff * sizeof(float4);
  const size_t ldse = tab + (256 + kGemmWaves * 64 * 3) * sizeof(float);
  const size_t ldsp = std::max(tab + 2 * a.pro_F * sizeof(float), ldse);
#define LAUNCH(P, E, L) hipLaunchKernelGGL((gemm_bs_kernel<P, E>), dim3(grid), dim3(64 * kGemmWaves), L, s, a)
#define LAUNCHK(P, E, K, L) hipLaunchKernelGGL((gemm_bs_kernel<P, E, K>), dim3(grid), dim3(64 * kGemmWaves), L, s, a)
  if (a.k_groups == 5 || a.k_groups == 7) {  // the lift: raw operand, BN statistics or none
    const bool k5 = a.k_groups == 5;
    if (a.epi_mode == EPI_BNFWD) { if (k5) LAUNCHK(PRO_RAW, EPI_BNFWD, 5, ldse); else LAUNCHK(PRO_RAW, EPI_BNFWD, 7, ldse); }
    else { if (k5) LAUNCHK(PRO_RAW, EPI_NONE, 5, lds); else LAUNCHK(PRO_RAW, EPI_NONE, 7, lds); }
  } else if (a.pro_mode == PRO_BNACT) {
    if (a.epi_mode == EPI_BNFWD) LAUNCH(PRO_BNACT, EPI_BNFWD, ldsp);
    else LAUNCH(PRO_BNACT, EPI_NONE, ldsp);
  } else {
    if (a.epi_mode == EPI_BNFWD) LAUNCH(PRO_RAW, EPI_BNFWD, ldse);
    else if (a.epi_mode == EPI_BNBACK && a.epi_drop.rate > 0.f) LAUNCH(PRO_RAW, kEpiBnBackDrop, ldse);
    else if (a.epi_mode == EPI_BNBACK) LAUNCH(PRO_RAW, EPI_BNBACK, ldse);
    else LAUNCH(PRO_RAW, EPI_NONE, lds);
  }
#undef LAUNCH
#undef LAUNCHK
#undef UIDX
}

}  // namespace lcn
