// Weight-gradient GEMM of the LCN hidden layers (gfx950): for every present
// 64x64 block (si, so), dW_e = A[:, si-slab]^T . dZ[:, so-slab] summed over
// the batch (the dW half of the autodiff of models_att.py:662, :692).  The
// batch is split into chunks; each chunk writes a partial slab that
// dw_reduce sums in a fixed order (deterministic, no atomics).
#include "gemm_common.h"

namespace lcn {

// dWe partials.  One workgroup = one 64x64 block (si, so) x one batch chunk;
// 4 waves in a 2x2 grid of 32x32 MFMA tiles; 64 batch rows per LDS stage.
// Work ids are chunk-major so the blocks of one chunk (same batch rows) run
// on one XCD and share A / dZ slabs through its L2.
// PRO: A operand gets BN apply + LeakyReLU; DBB: the D operand is dz rebuilt
// from (dh, z) by the BN + LeakyReLU backward, dz = c1 du + c2 + c3 z; the
// workgroups of one designated block per output slab also store that dz
// (dz_out) for the backward-data GEMM that follows, so dz costs one write and
// no separate elementwise pass.
template <bool PRO, bool DBB>
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
  BnBackCoef dcf{};
  if constexpr (DBB) {
    const int ch = (sb.y % a.spj_in) * kSlab + 4 * c4;
    dcf = load_bnback_coef(a.d_scale, a.d_shift, a.d_c123, a.d_F, ch);
  }
  const float* asrc = a.A + (size_t)sb.x * kSlab + 4 * c4;
  const float* dsrc = a.D + (size_t)sb.y * kSlab + 4 * c4;
  const float* zsrc = DBB ? a.d_z + (size_t)sb.y * kSlab + 4 * c4 : nullptr;
  const int glda = a.lda, gldd = a.ldd;
  float4 ra0, ra1, ra2, ra3, rd0, rd1, rd2, rd3, rz0, rz1, rz2, rz3;
  // rows >= r1 are clamped for the load; their D operand is zeroed when staged
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
    if constexpr (DBB) {                                                            \
      rz0 = *(const float4*)(zsrc + (size_t)c0_ * gldd);                            \
      rz1 = *(const float4*)(zsrc + (size_t)c1_ * gldd);                            \
      rz2 = *(const float4*)(zsrc + (size_t)c2_ * gldd);                            \
      rz3 = *(const float4*)(zsrc + (size_t)c3_ * gldd);                            \
    }                                                                               \
  }
  if (r0 < r1) DW_GLOAD(r0);
  for (int base = r0; base < r1; base += 64) {
    __syncthreads();
    if constexpr (PRO) {
      ra0 = bnact4(ra0, sc, sh, a.alpha); ra1 = bnact4(ra1, sc, sh, a.alpha);
      ra2 = bnact4(ra2, sc, sh, a.alpha); ra3 = bnact4(ra3, sc, sh, a.alpha);
    }
    if constexpr (DBB) {  // D = dz rebuilt from (dh, z) of the layer
      rd0 = bnback4(rd0, rz0, dcf, a.alpha); rd1 = bnback4(rd1, rz1, dcf, a.alpha);
      rd2 = bnback4(rd2, rz2, dcf, a.alpha); rd3 = bnback4(rd3, rz3, dcf, a.alpha);
    }
    {
      const int q0 = base + rr;
      const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q0 >= r1) rd0 = z4;
      if (q0 + 16 >= r1) rd1 = z4;
      if (q0 + 32 >= r1) rd2 = z4;
      if (q0 + 48 >= r1) rd3 = z4;
    }
    if constexpr (DBB) {  // one block per output slab writes dz for the dX GEMM
      if (a.dz_out && a.dz_writer[b]) {
        const int q0 = base + rr;
        float* o = a.dz_out + (size_t)sb.y * kSlab + 4 * c4;
        if (q0 < r1) *(float4*)(o + (size_t)q0 * gldd) = rd0;
        if (q0 + 16 < r1) *(float4*)(o + (size_t)(q0 + 16) * gldd) = rd1;
        if (q0 + 32 < r1) *(float4*)(o + (size_t)(q0 + 32) * gldd) = rd2;
        if (q0 + 48 < r1) *(float4*)(o + (size_t)(q0 + 48) * gldd) = rd3;
      }
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
  const bool pro = a.pro_scale != nullptr, dbb = a.d_bnback != 0;
  if (pro && dbb)
    hipLaunchKernelGGL((gemm_dw_kernel<true, true>), dim3(grid), dim3(256), lds, s, a);
  else if (pro)
    hipLaunchKernelGGL((gemm_dw_kernel<true, false>), dim3(grid), dim3(256), lds, s, a);
  else if (dbb)
    hipLaunchKernelGGL((gemm_dw_kernel<false, true>), dim3(grid), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL((gemm_dw_kernel<false, false>), dim3(grid), dim3(256), lds, s, a);
}

// Sum the chunk partials of every block in a fixed order and scatter into the
// dense gradient dW[rows][ld]; rows / columns past (rows_valid, cols_valid)
// are the zero padding of the thin lift / output layers and are dropped.
__global__ __launch_bounds__(256) void dw_reduce_kernel(const float* __restrict__ part, int nchunks,
                                                        int nblk, const int2* __restrict__ blk,
                                                        float* __restrict__ dW, int ld,
                                                        int rows_valid, int cols_valid) {
  const int b = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;  // 0..4095
  const int2 sb = blk[b];
  const int row = sb.x * kSlab + (e >> 6), col = sb.y * kSlab + (e & 63);
  if (row >= rows_valid || col >= cols_valid) return;
  const size_t stride = (size_t)nblk * 4096;
  const float* p = part + (size_t)b * 4096 + e;
  float s = 0.f;
  for (int c = 0; c < nchunks; ++c) s += p[c * stride];
  dW[(size_t)row * ld + col] = s;
}

void launch_dw_reduce(const float* part, int nchunks, int nblk, const int2* blk, float* dW, int ld,
                      int rows_valid, int cols_valid, hipStream_t s) {
  hipLaunchKernelGGL(dw_reduce_kernel, dim3(16, nblk), dim3(256), 0, s, part, nchunks, nblk, blk,
                     dW, ld, rows_valid, cols_valid);
}

}  // namespace lcn
