// Block-sparse fp32 MFMA GEMM of the LCN hidden layers, forward and
// backward-data (gfx950).
//
// Replaces the TF MatMul ops of cgcnn.two_linear (models_att.py:662, :692)
// and the dX half of their autodiff.  W_e = clip(W) (.) M (models_att.py:
// 576-586) is zero outside the blocks (i, j) with M[i,j] != 0, so a 64x64
// feature block of a joint pair is the unit of work and absent blocks are
// skipped (175 of 289 present at knn=3).  Output slab `so` of a row tile
// accumulates X[:, si-slab] . block over the CSR list ptr[so]..ptr[so+1].
//
// Exact fp32: v_mfma_f32_32x32x2_f32 (gfx950 has no xf32; the f32-input MFMA
// is a k-ordered fmaf chain).  32x32x2 operand map: lane l supplies A[i=l&31]
// [k=l>>5] and B[k=l>>5][j=l&31].  The k order inside each group of 8 is
// permuted -- lane half h takes k = 8g + 4h + s at step s -- so a lane's 4
// consecutive k-steps are 16 contiguous bytes of both operands.
#include "gemm_common.h"

namespace lcn {

// ---------------------------------------------------------------------------
// v0: 128 rows x 64 columns per workgroup, 4 waves of 32 rows x 64 columns;
// the 128x64 activation tile and the 64x64 weight block both staged in LDS
// (single buffer, register prefetch of the next slab; 3 workgroups per CU).
// ---------------------------------------------------------------------------
template <bool PRO>
__global__ __launch_bounds__(256) void gemm_bs_v0(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                  // [128][LDA]
  float* Ws = smem + 128 * LDA;      // [64][LDA]
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = wg / a.n_out_slabs, so = wg - rt * a.n_out_slabs;
  const int row0 = rt * 128;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c4 = t & 15, rr = t >> 4;
  const int lr = lane & 31, h = lane >> 5;
  const int beg = a.ptr[so], end = a.ptr[so + 1];

  f32x16 acc0, acc1;
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; }

  // named staging registers (arrays were demoted to scratch by the compiler)
  float4 ra0, ra1, ra2, ra3, ra4, ra5, ra6, ra7, rw0, rw1, rw2, rw3;
  const int2* __restrict__ gidx = a.idx;
  const float* __restrict__ gX = a.X;
  const float* __restrict__ gblocks = a.blocks;
  const int glast = a.B - 1, gldx = a.ldx;
  // rows past B are clamped, not zeroed: output rows are independent and
  // rows >= B are neither stored nor counted in the BN partials
#define V0_GLOAD(E)                                                                       \
  {                                                                                       \
    const int2 ib_ = gidx[(E)];                                                           \
    si_next = ib_.x;                                                                      \
    const float* src_ = gX + (size_t)ib_.x * kSlab + 4 * c4;                              \
    ra0 = *(const float4*)(src_ + (size_t)min(row0 + rr, glast) * gldx);                  \
    ra1 = *(const float4*)(src_ + (size_t)min(row0 + rr + 16, glast) * gldx);             \
    ra2 = *(const float4*)(src_ + (size_t)min(row0 + rr + 32, glast) * gldx);             \
    ra3 = *(const float4*)(src_ + (size_t)min(row0 + rr + 48, glast) * gldx);             \
    ra4 = *(const float4*)(src_ + (size_t)min(row0 + rr + 64, glast) * gldx);             \
    ra5 = *(const float4*)(src_ + (size_t)min(row0 + rr + 80, glast) * gldx);             \
    ra6 = *(const float4*)(src_ + (size_t)min(row0 + rr + 96, glast) * gldx);             \
    ra7 = *(const float4*)(src_ + (size_t)min(row0 + rr + 112, glast) * gldx);            \
    const float* wsrc_ = gblocks + (size_t)ib_.y * (kSlab * kSlab) + rr * kSlab + 4 * c4; \
    rw0 = *(const float4*)(wsrc_);                                                        \
    rw1 = *(const float4*)(wsrc_ + 16 * kSlab);                                           \
    rw2 = *(const float4*)(wsrc_ + 32 * kSlab);                                           \
    rw3 = *(const float4*)(wsrc_ + 48 * kSlab);                                           \
  }

  int si_next = 0;
  V0_GLOAD(beg);  // every output slab has >= 1 input block (checked in lcn_create)
  for (int e = beg; e < end; ++e) {
    const int si = si_next;
    __syncthreads();
    if constexpr (PRO) {
      const int ch = (si % a.spj_in) * kSlab + 4 * c4;
      const float4 sc = *(const float4*)(a.pro_scale + ch);
      const float4 sh = *(const float4*)(a.pro_shift + ch);
      const float al = a.alpha;
      ra0 = bnact4(ra0, sc, sh, al); ra1 = bnact4(ra1, sc, sh, al);
      ra2 = bnact4(ra2, sc, sh, al); ra3 = bnact4(ra3, sc, sh, al);
      ra4 = bnact4(ra4, sc, sh, al); ra5 = bnact4(ra5, sc, sh, al);
      ra6 = bnact4(ra6, sc, sh, al); ra7 = bnact4(ra7, sc, sh, al);
    }
    {
      float* ad = As + rr * LDA + 4 * c4;
      *(float4*)(ad) = ra0;
      *(float4*)(ad + 16 * LDA) = ra1;
      *(float4*)(ad + 32 * LDA) = ra2;
      *(float4*)(ad + 48 * LDA) = ra3;
      *(float4*)(ad + 64 * LDA) = ra4;
      *(float4*)(ad + 80 * LDA) = ra5;
      *(float4*)(ad + 96 * LDA) = ra6;
      *(float4*)(ad + 112 * LDA) = ra7;
      float* wd = Ws + rr * LDA + 4 * c4;
      *(float4*)(wd) = rw0;
      *(float4*)(wd + 16 * LDA) = rw1;
      *(float4*)(wd + 32 * LDA) = rw2;
      *(float4*)(wd + 48 * LDA) = rw3;
    }
    __syncthreads();
    if (e + 1 < end) V0_GLOAD(e + 1);

    const float* Ap = As + (32 * w + lr) * LDA + 4 * h;
    const float* B0 = Ws + lr * LDA + 4 * h;
    const float* B1 = Ws + (32 + lr) * LDA + 4 * h;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const float4 av = *(const float4*)(Ap + 8 * g);
      const float4 b0 = *(const float4*)(B0 + 8 * g);
      const float4 b1 = *(const float4*)(B1 + 8 * g);
      MFMA_STEP4(av, b0, b1, acc0, acc1);
    }
  }
#undef V0_GLOAD
  gemm_epilogue_32x64(a, acc0, acc1, rt, so, row0, w, lr, h, smem);
}

// ---------------------------------------------------------------------------
// v1: the same 128 x 64 tile, but every wave reads its own 32 activation rows
// straight into MFMA A-fragment registers (each activation element is used by
// exactly one wave, so LDS staging buys nothing for it); only the 64x64
// weight block, shared by the 4 waves, goes through LDS, double-buffered:
// one barrier per input slab, 35 KB of LDS -> 4 workgroups per CU.
// ---------------------------------------------------------------------------
template <bool PRO>
__global__ __launch_bounds__(256) void gemm_bs_v1(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int WBUF = 64 * LDA;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = wg / a.n_out_slabs, so = wg - rt * a.n_out_slabs;
  const int row0 = rt * 128;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c4 = t & 15, rr = t >> 4;
  const int lr = lane & 31, h = lane >> 5;
  const int beg = a.ptr[so], end = a.ptr[so + 1];

  f32x16 acc0, acc1;
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; }

  const int2* __restrict__ gidx = a.idx;
  const float* __restrict__ gblocks = a.blocks;
  // this lane's activation row (clamped: rows >= B are never stored or counted)
  const float* arow = a.X + (size_t)min(row0 + 32 * w + lr, a.B - 1) * a.ldx + 4 * h;
  float4 c0, c1, c2, c3, c4v, c5, c6, c7;   // current slab's A fragments (k = 8g + 4h + s)
  float4 n0, n1, n2, n3, n4, n5, n6, n7;    // next slab's
  float4 rw0, rw1, rw2, rw3;                // next weight block (staging)
  int si_cur = 0, si_nxt = 0;
#define V1_ALOAD(E, D0, D1, D2, D3, D4, D5, D6, D7, SI)   \
  {                                                       \
    const int2 ib_ = gidx[(E)];                           \
    SI = ib_.x;                                           \
    const float* p_ = arow + (size_t)ib_.x * kSlab;       \
    D0 = *(const float4*)(p_);                            \
    D1 = *(const float4*)(p_ + 8);                        \
    D2 = *(const float4*)(p_ + 16);                       \
    D3 = *(const float4*)(p_ + 24);                       \
    D4 = *(const float4*)(p_ + 32);                       \
    D5 = *(const float4*)(p_ + 40);                       \
    D6 = *(const float4*)(p_ + 48);                       \
    D7 = *(const float4*)(p_ + 56);                       \
    const float* w_ = gblocks + (size_t)ib_.y * (kSlab * kSlab) + rr * kSlab + 4 * c4; \
    rw0 = *(const float4*)(w_);                           \
    rw1 = *(const float4*)(w_ + 16 * kSlab);              \
    rw2 = *(const float4*)(w_ + 32 * kSlab);              \
    rw3 = *(const float4*)(w_ + 48 * kSlab);              \
  }
#define V1_WSTORE(BUFP)                                   \
  {                                                       \
    float* wd_ = (BUFP) + rr * LDA + 4 * c4;              \
    *(float4*)(wd_) = rw0;                                \
    *(float4*)(wd_ + 16 * LDA) = rw1;                     \
    *(float4*)(wd_ + 32 * LDA) = rw2;                     \
    *(float4*)(wd_ + 48 * LDA) = rw3;                     \
  }

  V1_ALOAD(beg, c0, c1, c2, c3, c4v, c5, c6, c7, si_cur);
  V1_WSTORE(smem);
  __syncthreads();
  for (int e = beg; e < end; ++e) {
    const int cur = (e - beg) & 1;
    V1_ALOAD(min(e + 1, end - 1), n0, n1, n2, n3, n4, n5, n6, n7, si_nxt);
    if constexpr (PRO) {
      // channel of k = 8g + 4h + s: ((si % spj) * 64 + 8g + 4h + s)
      const float* scp = a.pro_scale + (si_cur % a.spj_in) * kSlab + 4 * h;
      const float* shp = a.pro_shift + (si_cur % a.spj_in) * kSlab + 4 * h;
      const float al = a.alpha;
      c0 = bnact4(c0, *(const float4*)(scp), *(const float4*)(shp), al);
      c1 = bnact4(c1, *(const float4*)(scp + 8), *(const float4*)(shp + 8), al);
      c2 = bnact4(c2, *(const float4*)(scp + 16), *(const float4*)(shp + 16), al);
      c3 = bnact4(c3, *(const float4*)(scp + 24), *(const float4*)(shp + 24), al);
      c4v = bnact4(c4v, *(const float4*)(scp + 32), *(const float4*)(shp + 32), al);
      c5 = bnact4(c5, *(const float4*)(scp + 40), *(const float4*)(shp + 40), al);
      c6 = bnact4(c6, *(const float4*)(scp + 48), *(const float4*)(shp + 48), al);
      c7 = bnact4(c7, *(const float4*)(scp + 56), *(const float4*)(shp + 56), al);
    }
    const float* Wc = smem + cur * WBUF;
    const float* B0 = Wc + lr * LDA + 4 * h;
    const float* B1 = Wc + (32 + lr) * LDA + 4 * h;
#define V1_G(G, AV)                                       \
    {                                                     \
      const float4 b0 = *(const float4*)(B0 + 8 * (G));   \
      const float4 b1 = *(const float4*)(B1 + 8 * (G));   \
      MFMA_STEP4(AV, b0, b1, acc0, acc1);                 \
    }
    V1_G(0, c0) V1_G(1, c1) V1_G(2, c2) V1_G(3, c3)
    V1_G(4, c4v) V1_G(5, c5) V1_G(6, c6) V1_G(7, c7)
#undef V1_G
    V1_WSTORE(smem + (cur ^ 1) * WBUF);  // the last one is dead (unconditional: no scratch)
    __syncthreads();
    c0 = n0; c1 = n1; c2 = n2; c3 = n3; c4v = n4; c5 = n5; c6 = n6; c7 = n7;
    si_cur = si_nxt;
  }
#undef V1_ALOAD
#undef V1_WSTORE
  gemm_epilogue_32x64(a, acc0, acc1, rt, so, row0, w, lr, h, smem);
}

// ---------------------------------------------------------------------------
// v2: 256 rows x 64 columns per workgroup; each of the 4 waves owns 64 rows x
// 64 columns (2 x 2 accumulators), reads its activation fragments straight
// into registers (prefetching the next slab's) and shares the 64x64 weight
// block through a double-buffered LDS image (one barrier per input slab).
// Twice the MFMA work per barrier and per staged weight byte of v0/v1.
// ---------------------------------------------------------------------------
template <bool PRO>
__global__ __launch_bounds__(256, 2) void gemm_bs_v2(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int WBUF = 64 * LDA;
  float* sct = smem + 2 * WBUF;            // BN scale / shift tables [F] (PRO)
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = wg / a.n_out_slabs, so = wg - rt * a.n_out_slabs;
  const int row0 = rt * 256;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c4 = t & 15, rr = t >> 4;
  const int lr = lane & 31, h = lane >> 5;
  const int beg = a.ptr[so], end = a.ptr[so + 1];
  const int F = a.spj_in * kSlab;
  if constexpr (PRO) {
    for (int i = t; i < F; i += 256) { sct[i] = a.pro_scale[i]; sct[F + i] = a.pro_shift[i]; }
  }

  f32x16 acc00, acc01, acc10, acc11;
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc00[k] = 0.f; acc01[k] = 0.f; acc10[k] = 0.f; acc11[k] = 0.f; }

  const int2* __restrict__ gidx = a.idx;
  const float* __restrict__ gblocks = a.blocks;
  const int r0 = min(row0 + 64 * w + lr, a.B - 1), r1 = min(row0 + 64 * w + 32 + lr, a.B - 1);
  const float* arow0 = a.X + (size_t)r0 * a.ldx + 4 * h;
  const float* arow1 = a.X + (size_t)r1 * a.ldx + 4 * h;
  float4 x00, x01, x02, x03, x04, x05, x06, x07, x10, x11, x12, x13, x14, x15, x16, x17;
  float4 y00, y01, y02, y03, y04, y05, y06, y07, y10, y11, y12, y13, y14, y15, y16, y17;
  float4 rw0, rw1, rw2, rw3;
  int si_cur = 0, si_nxt = 0;
#define V2_ROW(P, D0, D1, D2, D3, D4, D5, D6, D7) \
  D0 = *(const float4*)(P);                       \
  D1 = *(const float4*)((P) + 8);                 \
  D2 = *(const float4*)((P) + 16);                \
  D3 = *(const float4*)((P) + 24);                \
  D4 = *(const float4*)((P) + 32);                \
  D5 = *(const float4*)((P) + 40);                \
  D6 = *(const float4*)((P) + 48);                \
  D7 = *(const float4*)((P) + 56);
#define V2_LOAD(E, X)                                                                     \
  {                                                                                       \
    const int2 ib_ = gidx[(E)];                                                           \
    si_nxt = ib_.x;                                                                       \
    const float* p0_ = arow0 + (size_t)ib_.x * kSlab;                                     \
    const float* p1_ = arow1 + (size_t)ib_.x * kSlab;                                     \
    V2_ROW(p0_, X##00, X##01, X##02, X##03, X##04, X##05, X##06, X##07)                   \
    V2_ROW(p1_, X##10, X##11, X##12, X##13, X##14, X##15, X##16, X##17)                   \
    const float* w_ = gblocks + (size_t)ib_.y * (kSlab * kSlab) + rr * kSlab + 4 * c4;   \
    rw0 = *(const float4*)(w_);                                                           \
    rw1 = *(const float4*)(w_ + 16 * kSlab);                                              \
    rw2 = *(const float4*)(w_ + 32 * kSlab);                                              \
    rw3 = *(const float4*)(w_ + 48 * kSlab);                                              \
  }
#define V2_WSTORE(BUFP)                                   \
  {                                                       \
    float* wd_ = (BUFP) + rr * LDA + 4 * c4;              \
    *(float4*)(wd_) = rw0;                                \
    *(float4*)(wd_ + 16 * LDA) = rw1;                     \
    *(float4*)(wd_ + 32 * LDA) = rw2;                     \
    *(float4*)(wd_ + 48 * LDA) = rw3;                     \
  }

  V2_LOAD(beg, x);
  si_cur = si_nxt;
  V2_WSTORE(smem);
  __syncthreads();
  for (int e = beg; e < end; ++e) {
    const int cur = (e - beg) & 1;
    V2_LOAD(min(e + 1, end - 1), y);
    const float* Wc = smem + cur * WBUF;
    const float* B0 = Wc + lr * LDA + 4 * h;
    const float* B1 = Wc + (32 + lr) * LDA + 4 * h;
    const float* scp = sct + (si_cur % a.spj_in) * kSlab + 4 * h;
    const float al = a.alpha;
#define V2_G(G, A0, A1)                                                        \
    {                                                                          \
      float4 a0_ = A0, a1_ = A1;                                               \
      if constexpr (PRO) {                                                     \
        const float4 sc_ = *(const float4*)(scp + 8 * (G));                    \
        const float4 sh_ = *(const float4*)(scp + F + 8 * (G));                \
        a0_ = bnact4(a0_, sc_, sh_, al);                                       \
        a1_ = bnact4(a1_, sc_, sh_, al);                                       \
      }                                                                        \
      const float4 b0 = *(const float4*)(B0 + 8 * (G));                        \
      const float4 b1 = *(const float4*)(B1 + 8 * (G));                        \
      MFMA_STEP4(a0_, b0, b1, acc00, acc01);                                   \
      MFMA_STEP4(a1_, b0, b1, acc10, acc11);                                   \
    }
    V2_G(0, x00, x10) V2_G(1, x01, x11) V2_G(2, x02, x12) V2_G(3, x03, x13)
    V2_G(4, x04, x14) V2_G(5, x05, x15) V2_G(6, x06, x16) V2_G(7, x07, x17)
#undef V2_G
    V2_WSTORE(smem + (cur ^ 1) * WBUF);  // the last one is dead (unconditional: no scratch)
    __syncthreads();
    x00 = y00; x01 = y01; x02 = y02; x03 = y03; x04 = y04; x05 = y05; x06 = y06; x07 = y07;
    x10 = y10; x11 = y11; x12 = y12; x13 = y13; x14 = y14; x15 = y15; x16 = y16; x17 = y17;
    si_cur = si_nxt;
  }
#undef V2_ROW
#undef V2_LOAD
#undef V2_WSTORE
  // epilogue: two 32-row halves of the wave, each as a 32x64 tile
  gemm_epilogue_64x64(a, acc00, acc01, acc10, acc11, rt, so, row0, w, lr, h, smem);
}

int gemm_bs_rows(int variant) { return variant == 2 ? 256 : 128; }

void launch_gemm_bs(const GemmArgs& a, hipStream_t s) {
  const int grid = ((a.B + gemm_bs_rows(a.variant) - 1) / gemm_bs_rows(a.variant)) * a.n_out_slabs;
  if (a.variant == 2) {
    const size_t lds = ((size_t)2 * 64 * LDA + 2 * a.spj_in * kSlab) * sizeof(float);
    if (a.pro_scale) hipLaunchKernelGGL(gemm_bs_v2<true>, dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL(gemm_bs_v2<false>, dim3(grid), dim3(256), lds, s, a);
  } else if (a.variant == 0) {
    const size_t lds = (size_t)(128 + 64) * LDA * sizeof(float);
    if (a.pro_scale) hipLaunchKernelGGL(gemm_bs_v0<true>, dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL(gemm_bs_v0<false>, dim3(grid), dim3(256), lds, s, a);
  } else {
    const size_t lds = (size_t)2 * 64 * LDA * sizeof(float);
    if (a.pro_scale) hipLaunchKernelGGL(gemm_bs_v1<true>, dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL(gemm_bs_v1<false>, dim3(grid), dim3(256), lds, s, a);
  }
}

}  // namespace lcn
