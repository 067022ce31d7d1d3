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
// is a k-ordered fmaf chain).  32x32x2 operand map: lane l supplies A[i=l&31]
// [k=l>>5] and B[k=l>>5][j=l&31].  The k order inside each group of 8 is
// permuted -- lane half h takes k = 8g + 4h + s at step s -- so a lane's 4
// consecutive k-steps are 16 contiguous bytes of both operands.
//
// Tile: 128 rows x 64 columns per workgroup, 4 waves of 32 rows x 64 columns
// (two 32x32 accumulators); the 128x64 activation tile and the 64x64 weight
// block are staged in LDS (row stride 68 floats: conflict-free ds_read_b128),
// the next input slab is prefetched into registers while the MFMAs run; 3
// workgroups per CU.  (Variants with register-resident A fragments, 256-row
// tiles or double-buffered LDS measured equal or slower: DESIGN.md §3.)
//
// Operand prologue (PRO), applied while staging the activation tile:
//   PRO_RAW     a = X
//   PRO_BNACT   a = leaky(scale * X + shift)                  (BN apply + LeakyReLU)
// (Rebuilding the backward's dz = c1 du + c2 + c3 z here was measured 27%
// slower than reading a stored dz: every input slab is re-staged by ~10
// output slabs, so the rebuild and the extra z stream are paid ~10 times;
// the weight-gradient kernel stores dz instead)
// Epilogue: + bias / + residual, store; then either BN forward partials of the
// output (sum, M2 about the tile mean) or BN backward partials of the layer
// below (sum du, sum du * zhat), per column of the 128-row tile.
#include "gemm_common.h"

namespace lcn {

template <int PRO>
__global__ __launch_bounds__(256) void gemm_bs_kernel(GemmArgs a) {
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
#define GL_ROWS(P, D0, D1, D2, D3, D4, D5, D6, D7)                         \
  D0 = *(const float4*)((P) + (size_t)min(row0 + rr, glast) * gldx);       \
  D1 = *(const float4*)((P) + (size_t)min(row0 + rr + 16, glast) * gldx);  \
  D2 = *(const float4*)((P) + (size_t)min(row0 + rr + 32, glast) * gldx);  \
  D3 = *(const float4*)((P) + (size_t)min(row0 + rr + 48, glast) * gldx);  \
  D4 = *(const float4*)((P) + (size_t)min(row0 + rr + 64, glast) * gldx);  \
  D5 = *(const float4*)((P) + (size_t)min(row0 + rr + 80, glast) * gldx);  \
  D6 = *(const float4*)((P) + (size_t)min(row0 + rr + 96, glast) * gldx);  \
  D7 = *(const float4*)((P) + (size_t)min(row0 + rr + 112, glast) * gldx);
#define GLOAD(E)                                                                          \
  {                                                                                       \
    const int2 ib_ = gidx[(E)];                                                           \
    si_next = ib_.x;                                                                      \
    const float* src_ = gX + (size_t)ib_.x * kSlab + 4 * c4;                              \
    GL_ROWS(src_, ra0, ra1, ra2, ra3, ra4, ra5, ra6, ra7)                                 \
    const float* wsrc_ = gblocks + (size_t)ib_.y * (kSlab * kSlab) + rr * kSlab + 4 * c4; \
    rw0 = *(const float4*)(wsrc_);                                                        \
    rw1 = *(const float4*)(wsrc_ + 16 * kSlab);                                           \
    rw2 = *(const float4*)(wsrc_ + 32 * kSlab);                                           \
    rw3 = *(const float4*)(wsrc_ + 48 * kSlab);                                           \
  }

  int si_next = 0;
  GLOAD(beg);  // every output slab has >= 1 input block (checked in lcn_create)
  for (int e = beg; e < end; ++e) {
    const int si = si_next;
    __syncthreads();
    if constexpr (PRO == PRO_BNACT) {
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
    if (e + 1 < end) GLOAD(e + 1);

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
#undef GLOAD
#undef GL_ROWS
  gemm_epilogue_32x64(a, acc0, acc1, rt, so, row0, w, lr, h, smem);
}

int gemm_bs_rows(int variant) {
  (void)variant;
  return 128;
}

void launch_gemm_bs(const GemmArgs& a, hipStream_t s) {
  const int grid = ((a.B + 127) / 128) * a.n_out_slabs;
  const size_t lds = (size_t)(128 + 64) * LDA * sizeof(float);
  if (a.pro_mode == PRO_BNACT)
    hipLaunchKernelGGL(gemm_bs_kernel<PRO_BNACT>, dim3(grid), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL(gemm_bs_kernel<PRO_RAW>, dim3(grid), dim3(256), lds, s, a);
}

}  // namespace lcn
