// Block-sparse fp32 MFMA GEMMs of the LCN hidden layers (gfx950).
//
// Replaces the TF MatMul ops of cgcnn.two_linear (models_att.py:662, :692)
// and their autodiff (dX = dZ.We^T, dWe = A^T.dZ).  The masked weight
// W_e = clip(W) (.) M (models_att.py:576-586) is zero outside the blocks
// (i, j) with M[i,j] != 0, so each 64x64 feature block of a joint pair is a
// unit of work and absent blocks are skipped entirely (175 of 289 at knn=3).
//
// All arithmetic is exact fp32: v_mfma_f32_32x32x2_f32 (gfx950 has no
// xf32/TF32; the f32-input MFMA is a k-ordered fmaf chain).
#include "lcn_internal.h"

namespace lcn {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int LDA = 68;  // LDS row stride (floats): +4 breaks ds_read_b128 bank conflicts

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  // blocks b, b+8, ... share an XCD; give each XCD a contiguous range of work ids
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

__device__ __forceinline__ float leaky(float u, float alpha) { return u > 0.f ? u : u * alpha; }

__device__ __forceinline__ float4 bnact4(float4 v, float4 sc, float4 sh, float alpha) {
  v.x = leaky(fmaf(v.x, sc.x, sh.x), alpha);
  v.y = leaky(fmaf(v.y, sc.y, sh.y), alpha);
  v.z = leaky(fmaf(v.z, sc.z, sh.z), alpha);
  v.w = leaky(fmaf(v.w, sc.w, sh.w), alpha);
  return v;
}

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

// One workgroup = 128 batch rows x one 64-wide output slab.  4 waves, each
// 32 rows x 64 columns (two 32x32 accumulators).  Per input slab of the
// output slab's neighbour list: the 128x64 A tile and the 64x64 weight block
// are staged in LDS (register prefetch of the next slab overlaps the MFMAs).
// The k order inside a group of 8 is permuted (lane half h takes k = 8g+4h+s
// at step s) so every fragment read is one conflict-free ds_read_b128.
template <bool PRO>
__global__ __launch_bounds__(256) void gemm_bs_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                  // [128][LDA]
  float* Ws = smem + kGemmBM * LDA;  // [64][LDA]
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = wg / a.n_out_slabs, so = wg - rt * a.n_out_slabs;
  const int row0 = rt * kGemmBM;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c4 = t & 15, rr = t >> 4;
  const int lr = lane & 31, h = lane >> 5;
  const int beg = a.ptr[so], end = a.ptr[so + 1];

  f32x16 acc0, acc1;
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; }

  // Staging registers: named scalars (an array captured by a lambda or
  // indexed through a conditional load ended up in scratch).
  float4 ra0, ra1, ra2, ra3, ra4, ra5, ra6, ra7, rw0, rw1, rw2, rw3;
  const int2* __restrict__ gidx = a.idx;
  const float* __restrict__ gX = a.X;
  const float* __restrict__ gblocks = a.blocks;
  const int glast = a.B - 1, gldx = a.ldx;
  // rows past B are clamped, not zeroed: output rows are independent and
  // rows >= B are neither stored nor counted in the BN partials
#define GEMM_GLOAD(E)                                                                     \
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
  if (beg < end) GEMM_GLOAD(beg);
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
    if (e + 1 < end) GEMM_GLOAD(e + 1);
#undef GEMM_GLOAD

    const float* Ap = As + (32 * w + lr) * LDA + 4 * h;
    const float* B0 = Ws + lr * LDA + 4 * h;
    const float* B1 = Ws + (32 + lr) * LDA + 4 * h;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const float4 av = *(const float4*)(Ap + 8 * g);
      const float4 b0 = *(const float4*)(B0 + 8 * g);
      const float4 b1 = *(const float4*)(B1 + 8 * g);
      acc0 = MFMA32(av.x, b0.x, acc0);
      acc1 = MFMA32(av.x, b1.x, acc1);
      acc0 = MFMA32(av.y, b0.y, acc0);
      acc1 = MFMA32(av.y, b1.y, acc1);
      acc0 = MFMA32(av.z, b0.z, acc0);
      acc1 = MFMA32(av.z, b1.z, acc1);
      acc0 = MFMA32(av.w, b0.w, acc0);
      acc1 = MFMA32(av.w, b1.w, acc1);
    }
  }

  // Epilogue: C/D map of 32x32 MFMA: column = lane&31, row = (k&3) + 8(k>>2) + 4(lane>>5)
  const int ncol0 = so * kSlab + lr, ncol1 = ncol0 + 32;
  const float bias0 = a.bias ? a.bias[ncol0] : 0.f;
  const float bias1 = a.bias ? a.bias[ncol1] : 0.f;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int row = row0 + 32 * w + (k & 3) + 8 * (k >> 2) + 4 * h;
    float v0 = acc0[k] + bias0, v1 = acc1[k] + bias1;
    if (row < a.B) {
      const size_t o = (size_t)row * a.ldy;
      if (a.addsrc) { v0 += a.addsrc[o + ncol0]; v1 += a.addsrc[o + ncol1]; }
      a.Y[o + ncol0] = v0;
      a.Y[o + ncol1] = v1;
      s0 += v0;
      s1 += v1;
    }
    acc0[k] = v0;
    acc1[k] = v1;
  }
  if (a.stat == nullptr) return;
  // BN partials of this 128-row tile: (sum, sum of squares about the tile mean)
  const int nval = min(kGemmBM, a.B - row0);
  s0 += __shfl_xor(s0, 32);
  s1 += __shfl_xor(s1, 32);
  __syncthreads();
  float* red = smem;  // [4][64] sums, [4][64] m2
  if (h == 0) { red[w * 64 + lr] = s0; red[w * 64 + 32 + lr] = s1; }
  __syncthreads();
  const float tot0 = (red[lr] + red[64 + lr]) + (red[128 + lr] + red[192 + lr]);
  const float tot1 = (red[32 + lr] + red[96 + lr]) + (red[160 + lr] + red[224 + lr]);
  const float mean0 = tot0 / (float)nval, mean1 = tot1 / (float)nval;
  float m0 = 0.f, m1 = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int row = row0 + 32 * w + (k & 3) + 8 * (k >> 2) + 4 * h;
    if (row < a.B) {
      const float d0 = acc0[k] - mean0, d1 = acc1[k] - mean1;
      m0 = fmaf(d0, d0, m0);
      m1 = fmaf(d1, d1, m1);
    }
  }
  m0 += __shfl_xor(m0, 32);
  m1 += __shfl_xor(m1, 32);
  float* red2 = smem + 256;
  if (h == 0) { red2[w * 64 + lr] = m0; red2[w * 64 + 32 + lr] = m1; }
  __syncthreads();
  if (w == 0 && h == 0) {
    const float q0 = (red2[lr] + red2[64 + lr]) + (red2[128 + lr] + red2[192 + lr]);
    const float q1 = (red2[32 + lr] + red2[96 + lr]) + (red2[160 + lr] + red2[224 + lr]);
    a.stat[(size_t)rt * a.ldy + ncol0] = make_float2(tot0, q0);
    a.stat[(size_t)rt * a.ldy + ncol1] = make_float2(tot1, q1);
  }
}

void launch_gemm_bs(const GemmArgs& a, hipStream_t s) {
  const int grid = a.n_row_tiles * a.n_out_slabs;
  const size_t lds = (size_t)(kGemmBM + kSlab) * LDA * sizeof(float);
  if (a.pro_scale)
    hipLaunchKernelGGL(gemm_bs_kernel<true>, dim3(grid), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL(gemm_bs_kernel<false>, dim3(grid), dim3(256), lds, s, a);
}

// dWe partials.  One workgroup = one 64x64 block (si, so) x one batch chunk;
// 4 waves in a 2x2 grid of 32x32 MFMA tiles; 64 batch rows per LDS stage.
// Work ids are chunk-major so the blocks of one chunk (same batch rows) run
// on one XCD and share A / dZ slabs through its L2.
template <bool PRO>
__global__ __launch_bounds__(256) void gemm_dw_kernel(GemmDwArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;            // [64 rows][64 p]
  float* Ds = smem + 64 * 64;  // [64 rows][64 q]
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = wg / a.nblk, b = wg - chunk * a.nblk;
  const int2 sb = a.blk[b];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c4 = t & 15, rr = t >> 4;
  const int lr = lane & 31, h = lane >> 5;
  const int wp = w >> 1, wq = w & 1;
  const int r0 = chunk * a.chunk_rows;
  const int r1 = min(a.B, r0 + a.chunk_rows);

  f32x16 acc;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.f;

  float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sh = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (PRO) {
    const int ch = (sb.x % a.spj_in) * kSlab + 4 * c4;
    sc = *(const float4*)(a.pro_scale + ch);
    sh = *(const float4*)(a.pro_shift + ch);
  }
  const float* asrc = a.A + (size_t)sb.x * kSlab + 4 * c4;
  const float* dsrc = a.D + (size_t)sb.y * kSlab + 4 * c4;
  const int glda = a.lda, gldd = a.ldd;
  float4 ra0, ra1, ra2, ra3, rd0, rd1, rd2, rd3;
  // rows >= r1 are clamped for the load and zeroed by a select (no branches)
#define DW_GLOAD(BASE)                                                              \
  {                                                                                 \
    const int q0_ = (BASE) + rr;                                                    \
    const int c0_ = min(q0_, r1 - 1), c1_ = min(q0_ + 16, r1 - 1);                  \
    const int c2_ = min(q0_ + 32, r1 - 1), c3_ = min(q0_ + 48, r1 - 1);             \
    ra0 = *(const float4*)(asrc + (size_t)c0_ * glda);                              \
    ra1 = *(const float4*)(asrc + (size_t)c1_ * glda);                              \
    ra2 = *(const float4*)(asrc + (size_t)c2_ * glda);                              \
    ra3 = *(const float4*)(asrc + (size_t)c3_ * glda);                              \
    rd0 = *(const float4*)(dsrc + (size_t)c0_ * gldd);                              \
    rd1 = *(const float4*)(dsrc + (size_t)c1_ * gldd);                              \
    rd2 = *(const float4*)(dsrc + (size_t)c2_ * gldd);                              \
    rd3 = *(const float4*)(dsrc + (size_t)c3_ * gldd);                              \
    const float z4 = 0.f;                                                           \
    if (q0_ >= r1) rd0 = make_float4(z4, z4, z4, z4);                               \
    if (q0_ + 16 >= r1) rd1 = make_float4(z4, z4, z4, z4);                          \
    if (q0_ + 32 >= r1) rd2 = make_float4(z4, z4, z4, z4);                          \
    if (q0_ + 48 >= r1) rd3 = make_float4(z4, z4, z4, z4);                          \
  }
  if (r0 < r1) DW_GLOAD(r0);
  for (int base = r0; base < r1; base += 64) {
    __syncthreads();
    if constexpr (PRO) {
      ra0 = bnact4(ra0, sc, sh, a.alpha); ra1 = bnact4(ra1, sc, sh, a.alpha);
      ra2 = bnact4(ra2, sc, sh, a.alpha); ra3 = bnact4(ra3, sc, sh, a.alpha);
    }
    {
      float* ad = As + rr * 64 + 4 * c4;
      float* dd = Ds + rr * 64 + 4 * c4;
      *(float4*)(ad) = ra0;
      *(float4*)(ad + 16 * 64) = ra1;
      *(float4*)(ad + 32 * 64) = ra2;
      *(float4*)(ad + 48 * 64) = ra3;
      *(float4*)(dd) = rd0;
      *(float4*)(dd + 16 * 64) = rd1;
      *(float4*)(dd + 32 * 64) = rd2;
      *(float4*)(dd + 48 * 64) = rd3;
    }
    __syncthreads();
    if (base + 64 < r1) DW_GLOAD(base + 64);
#undef DW_GLOAD
    const float* Ap = As + 32 * wp + lr + 4 * h * 64;
    const float* Dp = Ds + 32 * wq + lr + 4 * h * 64;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float av = Ap[(8 * g + s) * 64];
        const float dv = Dp[(8 * g + s) * 64];
        acc = MFMA32(av, dv, acc);
      }
    }
  }
  float* out = a.part + ((size_t)chunk * a.nblk + b) * 4096;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int p = 32 * wp + (k & 3) + 8 * (k >> 2) + 4 * h;
    out[p * 64 + 32 * wq + lr] = acc[k];
  }
}

void launch_gemm_dw(const GemmDwArgs& a, hipStream_t s) {
  const int grid = a.nblk * a.nchunks;
  const size_t lds = 2 * 64 * 64 * sizeof(float);
  if (a.pro_scale)
    hipLaunchKernelGGL(gemm_dw_kernel<true>, dim3(grid), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL(gemm_dw_kernel<false>, dim3(grid), dim3(256), lds, s, a);
}

__global__ __launch_bounds__(256) void dw_reduce_kernel(const float* __restrict__ part, int nchunks,
                                                        int nblk, const int2* __restrict__ blk,
                                                        float* __restrict__ dW, int ld) {
  const int b = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;  // 0..4095
  const size_t stride = (size_t)nblk * 4096;
  const float* p = part + (size_t)b * 4096 + e;
  float s = 0.f;
  for (int c = 0; c < nchunks; ++c) s += p[c * stride];
  const int2 sb = blk[b];
  dW[(size_t)(sb.x * kSlab + (e >> 6)) * ld + sb.y * kSlab + (e & 63)] = s;
}

void launch_dw_reduce(const float* part, int nchunks, int nblk, const int2* blk, float* dW, int ld,
                      hipStream_t s) {
  hipLaunchKernelGGL(dw_reduce_kernel, dim3(16, nblk), dim3(256), 0, s, part, nchunks, nblk, blk,
                     dW, ld);
}

}  // namespace lcn
