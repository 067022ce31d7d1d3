// Block-sparse fp32 MFMA GEMM of the hidden LCN layers, forward and
// backward-data, TWO output slabs per workgroup (gfx950).
//
// Same contract as gemm_bs_kernel (gemm_bs.hip; tf.matmul of cgcnn.two_linear,
// models_att.py:662, :692, and the dX half of its autodiff), same operand
// layouts, same epilogues (gemm_epilogue.h).  What differs is the register
// tile: a wave owns one 32-row tile x a PAIR of 64-wide output slabs (four
// 32x32 accumulators) and walks the union of the two slabs' input lists; an
// input slab that both lists hold is loaded (and, for PRO_BNACT, transformed)
// once and multiplied by both weight blocks.  Beside a stream of MFMAs every
// operand load costs matrix-core time (scripts/microbench/mfma_steps.hip: the
// loop's 12 loads per 64 MFMAs 88.5 % of the fp32 MFMA peak, 93.7 % with the
// activation loads on every other block only), and the host pairs the output
// slabs by list overlap (make_pair_plan: 72 of 175 activation loads saved at
// knn 3, half of them when a joint has several slabs).
//
// The weight blocks still go through the double LDS buffer one block a step
// (LDS-DMA one step ahead, one barrier a step); the buffer index is a scalar
// that flips every step, the accumulator pair of a step is static (separate
// code per output slab of the pair).  168 VGPRs: three workgroups per CU.
#include <algorithm>

#include "gemm_epilogue.h"

namespace lcn {

#define STEP4(A0, A1, W0, W1, XV)    \
  A0 = MFMA32((W0).x, (XV).x, A0);   \
  A1 = MFMA32((W1).x, (XV).x, A1);   \
  A0 = MFMA32((W0).y, (XV).y, A0);   \
  A1 = MFMA32((W1).y, (XV).y, A1);   \
  A0 = MFMA32((W0).z, (XV).z, A0);   \
  A1 = MFMA32((W1).z, (XV).z, A1);   \
  A0 = MFMA32((W0).w, (XV).w, A0);   \
  A1 = MFMA32((W1).w, (XV).w, A1);
#define DECLX(P) float4 P##0, P##1, P##2, P##3, P##4, P##5, P##6, P##7;
// activation fragments of input slab SI (8 chunks of this wave's row tile)
#define LOADX(P, SI)                                                      \
  {                                                                       \
    const int so_ = (SI) * 8192;                                          \
    P##0 = BUFLD(xres, xlo, so_);          P##1 = BUFLD(xres, xlo + 1024, so_); \
    P##2 = BUFLD(xres, xlo + 2048, so_);   P##3 = BUFLD(xres, xlo + 3072, so_); \
    P##4 = BUFLD(xres, xlo, so_ + 4096);          P##5 = BUFLD(xres, xlo + 1024, so_ + 4096); \
    P##6 = BUFLD(xres, xlo + 2048, so_ + 4096);   P##7 = BUFLD(xres, xlo + 3072, so_ + 4096); \
  }
// this wave's quarter of weight block BLK, global -> LDS buffer BUF by LDS-DMA
#define GLDS(SOFF, DST) \
  __builtin_amdgcn_raw_ptr_buffer_load_lds(wres, (__attribute__((address_space(3))) void*)(DST), 16, xlo, (SOFF), 0, 0);
#define LOADW(BLK, BUF)                                                   \
  {                                                                       \
    const int bo_ = (BLK) * 16384 + wv_u * 1024;                          \
    float4* d_ = Wl + (BUF) * 1024 + wv_u * 64;                           \
    GLDS(bo_, d_) GLDS(bo_ + 4096, d_ + 256) GLDS(bo_ + 8192, d_ + 512) GLDS(bo_ + 12288, d_ + 768) \
  }
#define TSTEP(G, XV, CH)                                                  \
  {                                                                       \
    const int c_ = (CH) + 8 * (G) + 4 * h;                                \
    XV = bnact4(XV, *(const float4*)(tsc + c_), *(const float4*)(tsh + c_), al); \
  }
// BN apply + LeakyReLU of a slab's eight fragments, once per input slab (not
// once per weight block that multiplies it)
#define TRANSX(P, CH)                                                     \
  if constexpr (PRO == PRO_BNACT) {                                       \
    TSTEP(0, P##0, CH) TSTEP(1, P##1, CH) TSTEP(2, P##2, CH) TSTEP(3, P##3, CH) \
    TSTEP(4, P##4, CH) TSTEP(5, P##5, CH) TSTEP(6, P##6, CH) TSTEP(7, P##7, CH) \
    __builtin_amdgcn_sched_barrier(0);                                    \
  }
#define GSTEP(A0, A1, WB, G, XV)                                          \
  {                                                                       \
    const float4 w0_ = (WB)[(2 * (G)) * 64];                              \
    const float4 w1_ = (WB)[(2 * (G) + 1) * 64];                          \
    STEP4(A0, A1, w0_, w1_, XV)                                           \
  }
// schedule of one block: the LDS reads of group g+1 are issued before the 8
// MFMAs of group g, so their latency hides under those MFMAs
#define SGB(MASK, N) __builtin_amdgcn_sched_group_barrier(MASK, N, 0);
#define SCHED_SLAB                                                      \
  SGB(0x100, 2)                                                         \
  SGB(0x100, 2) SGB(0x008, 8) SGB(0x100, 2) SGB(0x008, 8)               \
  SGB(0x100, 2) SGB(0x008, 8) SGB(0x100, 2) SGB(0x008, 8)               \
  SGB(0x100, 2) SGB(0x008, 8) SGB(0x100, 2) SGB(0x008, 8)               \
  SGB(0x100, 2) SGB(0x008, 8) SGB(0x008, 8)
// one block step: 64 MFMAs of x set P against the block in LDS buffer `buf`
#define COMP(A0, A1, P)                                                   \
  {                                                                       \
    const float4* wb_ = Wl + buf * 1024 + lane;                           \
    GSTEP(A0, A1, wb_, 0, P##0) GSTEP(A0, A1, wb_, 1, P##1) GSTEP(A0, A1, wb_, 2, P##2) \
    GSTEP(A0, A1, wb_, 3, P##3) GSTEP(A0, A1, wb_, 4, P##4) GSTEP(A0, A1, wb_, 5, P##5) \
    GSTEP(A0, A1, wb_, 6, P##6) GSTEP(A0, A1, wb_, 7, P##7) SCHED_SLAB    \
  }
// merged list entry E: (input slab, block of slab A or -1, block of slab B or -1); wave-uniform
#define MENT(E)                                                           \
  ({                                                                      \
    const int4 t_ = ment[(E)];                                            \
    make_int4(__builtin_amdgcn_readfirstlane(t_.x), __builtin_amdgcn_readfirstlane(t_.y), \
              __builtin_amdgcn_readfirstlane(t_.z), 0);                   \
  })
// One merged entry EC (index EI), its activations in set P: the next entry's
// activations go into set Q and every step sends the following step's weight
// block into the other LDS buffer before it multiplies.  The barrier after a
// step drains that LDS-DMA (vmcnt(0)) and publishes it.
#define ENTRY(P, Q, EC, EN, EI)                                           \
  {                                                                       \
    const bool hn_ = (EI) + 1 < mend;                                     \
    int nfirst_ = -1;                                                     \
    if (hn_) {                                                            \
      EN = MENT((EI) + 1);                                                \
      nfirst_ = EN.y >= 0 ? EN.y : EN.z;                                  \
    }                                                                     \
    const int ch_ = (EC.x % spj) * kSlab;                                 \
    {                                                                     \
      const int nb_ = EC.y >= 0 && EC.z >= 0 ? EC.z : nfirst_;            \
      if (nb_ >= 0) LOADW(nb_, buf ^ 1)                                   \
    }                                                                     \
    if (hn_) LOADX(Q, EN.x)                                               \
    TRANSX(P, ch_)                                                        \
    if (EC.y >= 0) {                                                      \
      COMP(acc0, acc1, P)                                                 \
      __syncthreads();                                                    \
      buf ^= 1;                                                           \
      if (EC.z >= 0 && nfirst_ >= 0) LOADW(nfirst_, buf ^ 1)              \
    }                                                                     \
    if (EC.z >= 0) {                                                      \
      COMP(acc2, acc3, P)                                                 \
      __syncthreads();                                                    \
      buf ^= 1;                                                           \
    }                                                                     \
  }

// float offsets (from Wl + kTabOff) of the epilogue's LDS: table of slab A,
// the wave merge, table of slab B
constexpr int kPairComb = 256, kPairTabB = 256 + kGemmWaves * 64 * 3;

template <int PRO, int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void gemm_bs_pair_kernel(GemmArgs a) {
  static_assert(kGemmWaves == 4, "the pair kernel is built for four waves per workgroup");
  extern __shared__ __attribute__((aligned(16))) float4 Wl[];  // [2][1024] (+ BN tables)
  // Work map: as in gemm_bs_kernel, with pairs of output slabs in place of the
  // slabs.  Workgroups b, b + 8, ... share an XCD: each XCD walks a contiguous
  // range of row-tile groups, and the last `tail` groups of the range are
  // issued longest pair first (order[]).
  const int np = a.n_pairs;
  const int n_rtg = (a.n_rt + kGemmWaves - 1) / kGemmWaves;
  const int xcd = blockIdx.x & 7, li = blockIdx.x >> 3;
  const int base = n_rtg >> 3, extra = n_rtg & 7;
  const int g0 = xcd * base + min(xcd, extra), R = base + (xcd < extra ? 1 : 0);
  if (li >= R * np) return;  // padding of the grid (uniform per workgroup)
  const int T = a.pair_order ? min(R, a.tail) : 0;
  int rtg, pi;
  if (li < (R - T) * np) {
    rtg = li / np;
    pi = li - rtg * np;
    rtg += g0;
  } else {
    const int j = li - (R - T) * np, rank = j / T;
    pi = a.pair_order[rank];
    rtg = g0 + (R - T) + (j - rank * T);
  }
  const int4 pr = a.pairs[pi];
  const int soA = __builtin_amdgcn_readfirstlane(pr.x), soB = __builtin_amdgcn_readfirstlane(pr.y);
  const int mbeg = __builtin_amdgcn_readfirstlane(pr.z), mend = __builtin_amdgcn_readfirstlane(pr.w);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int wv_u = __builtin_amdgcn_readfirstlane(w);
  const int rt_raw = rtg * kGemmWaves + wv_u;
  const bool live = rt_raw < a.n_rt;
  // waves past the last row tile recompute it (they take part in the barriers)
  const int rt = live ? rt_raw : a.n_rt - 1;
  const int4* __restrict__ ment = a.ment;
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)a.X + (size_t)rt * a.S_in * 8192), 0, (a.S_in ? a.S_in : a.n_out_slabs) * 8192, 0x00020000);
  const __amdgpu_buffer_rsrc_t wres =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.blocks, 0, a.n_blocks * 16384, 0x00020000);
  const int xlo = lane * 16;  // the one address register of every operand load
  const float al = a.alpha;
  const float* tsc = nullptr;
  const float* tsh = nullptr;
  const int spj = a.spj_in;

  DECLX(xa)
  DECLX(xb)
  int4 ea = MENT(mbeg), eb = ea;
  int buf = 0;
  LOADW(ea.y >= 0 ? ea.y : ea.z, 0)
  LOADX(xa, ea.x)
  if constexpr (PRO == PRO_BNACT) {  // BN scale / shift of the operand's layer -> LDS
    float* tb = (float*)(Wl + kTabOff);
    for (int c = threadIdx.x; c < a.pro_F; c += 256) {
      tb[c] = a.pro_scale[c];
      tb[a.pro_F + c] = a.pro_shift[c];
    }
    tsc = tb;
    tsh = tb + a.pro_F;
  }
  float* etab = (float*)(Wl + kTabOff);
  if constexpr (EPI == EPI_BNBACK || EPI == kEpiBnBackDrop) {
    epi_fill_table(a, etab, soA);
    if (soB >= 0) epi_fill_table(a, etab + kPairTabB, soB);
  }
  // accumulators start at the bias (the MFMAs add onto it)
  f32x16 acc0, acc1, acc2, acc3;
  {
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 b0 = zero4, b1 = zero4, b2 = zero4, b3 = zero4;
      if (a.bias) {
        b0 = *(const float4*)(a.bias + soA * kSlab + 8 * q + 4 * h);
        b1 = *(const float4*)(a.bias + soA * kSlab + 8 * (4 + q) + 4 * h);
        if (soB >= 0) {
          b2 = *(const float4*)(a.bias + soB * kSlab + 8 * q + 4 * h);
          b3 = *(const float4*)(a.bias + soB * kSlab + 8 * (4 + q) + 4 * h);
        }
      }
      acc0[4 * q + 0] = b0.x; acc0[4 * q + 1] = b0.y; acc0[4 * q + 2] = b0.z; acc0[4 * q + 3] = b0.w;
      acc1[4 * q + 0] = b1.x; acc1[4 * q + 1] = b1.y; acc1[4 * q + 2] = b1.z; acc1[4 * q + 3] = b1.w;
      acc2[4 * q + 0] = b2.x; acc2[4 * q + 1] = b2.y; acc2[4 * q + 2] = b2.z; acc2[4 * q + 3] = b2.w;
      acc3[4 * q + 0] = b3.x; acc3[4 * q + 1] = b3.y; acc3[4 * q + 2] = b3.z; acc3[4 * q + 3] = b3.w;
    }
  }
  __syncthreads();
  // every pair has >= 1 merged entry (every output slab has an input block: lcn_create)
  for (int e = mbeg; e < mend; e += 2) {
    ENTRY(xa, xb, ea, eb, e)
    if (e + 1 < mend) ENTRY(xb, xa, eb, ea, e + 1)
  }

  // ---- epilogue: slab A, then slab B ----
  gemm_epilogue<EPI>(a, Wl, etab, etab + kPairComb, rtg, rt, live, soA, acc0, acc1);
  if (soB >= 0) gemm_epilogue<EPI>(a, Wl, etab + kPairTabB, etab + kPairComb, rtg, rt, live, soB, acc2, acc3);
}

void launch_gemm_bs_pair(const GemmArgs& a, hipStream_t s) {
  const int n_rtg = (a.n_rt + kGemmWaves - 1) / kGemmWaves;
  const int grid = 8 * ((n_rtg + 7) / 8) * a.n_pairs;  // 8 XCDs x row-tile groups per XCD x pairs
  // weight double buffer; BN tables / epilogue constants and the 4-wave merge after it
  const size_t lds = 2 * 1024 * sizeof(float4);
  const size_t tab = kTabOff * sizeof(float4);
  const size_t ldse = tab + (kPairTabB + 256) * sizeof(float);
  const size_t ldsp = std::max(tab + 2 * a.pro_F * sizeof(float), ldse);
#define LAUNCH(P, E, L) hipLaunchKernelGGL((gemm_bs_pair_kernel<P, E>), dim3(grid), dim3(256), L, s, a)
  if (a.pro_mode == PRO_BNACT) {
    if (a.epi_mode == EPI_BNFWD) LAUNCH(PRO_BNACT, EPI_BNFWD, ldsp);
    else LAUNCH(PRO_BNACT, EPI_NONE, ldsp);
  } else {
    if (a.epi_mode == EPI_BNFWD) LAUNCH(PRO_RAW, EPI_BNFWD, ldse);
    else if (a.epi_mode == EPI_BNBACK && a.epi_drop.rate > 0.f) LAUNCH(PRO_RAW, kEpiBnBackDrop, ldse);
    else if (a.epi_mode == EPI_BNBACK) LAUNCH(PRO_RAW, EPI_BNBACK, ldse);
    else LAUNCH(PRO_RAW, EPI_NONE, lds);
  }
#undef LAUNCH
}

}  // namespace lcn
