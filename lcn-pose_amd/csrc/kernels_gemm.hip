// Weight-gradient GEMM of the LCN layers (gfx950): for every present 64x64
// block (si, so), dW_e = A[:, si-slab]^T . dZ[:, so-slab] summed over the
// batch (the dW half of the autodiff of models_att.py:662, :692, and of the
// thin lift / output layers).  The batch is split into chunks; each chunk
// writes a partial slab that dw_reduce sums in a fixed order (deterministic,
// no atomics).
#include "gemm_common.h"

namespace lcn {

// One workgroup = one 64x64 block (si, so) x one batch chunk; 4 waves in a
// 2x2 grid of 32x32 MFMA tiles; 64 batch rows (two row tiles) per LDS stage.
// Work ids are chunk-major so the blocks of one chunk (same batch rows) run
// on one XCD and share the activation tiles through its L2.
//
// Staging: every thread loads 4 float4 of each operand's two 8 KB row-tile
// slabs (coalesced 1 KB chunks), applies the operand transform, and scatters
// them transposed into LDS ([feature][row], row stride 68 floats: the scatter
// and the ds_read_b128 fragment reads are both bank-conflict free).  The MFMA
// runs over the batch: lane l supplies A[b][p = l&31] and D[b][q = l&31] for
// k = b, four consecutive rows per float4 (lane half h takes rows 8g + 4h + s).
//
// PRO: the A operand gets BN apply + LeakyReLU (A = z of the layer below the
// block's inner layer); DBB: the D operand is dz rebuilt from (dh, z) by the
// BN + LeakyReLU backward, dz = c1 du + c2 + c3 z; the workgroups of one
// designated block per output slab also store that dz (dz_out) for the
// backward-data GEMM that follows, so dz costs one write and no separate
// elementwise pass.
constexpr int kDwLd = 68;

template <bool PRO, bool DBB>
__global__ __launch_bounds__(256) void gemm_dw_kernel(GemmDwArgs a) {
  __shared__ __attribute__((aligned(16))) float As[64 * kDwLd];  // [p][row]
  __shared__ __attribute__((aligned(16))) float Ds[64 * kDwLd];  // [q][row]
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = wg / a.nblk, b = wg - chunk * a.nblk;
  const int2 sb = a.blk[b];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int lr = lane & 31, h = lane >> 5;
  const int wp = w >> 1, wq = w & 1;
  const int r0 = chunk * a.chunk_rows;
  const int r1 = min(a.B, r0 + a.chunk_rows);
  const int last_rt = (a.B + kRT - 1) / kRT - 1;
  const bool writer = DBB && a.dz_out && a.dz_writer[b];

  f32x16 acc;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.f;

  // this thread's staging slots: j = 0..3 -> row tile j >> 1 of the stage,
  // chunk g = w + 4 (j & 1), lane `lane`: features 8g + 4h .. +3
  float4 sc0 = make_float4(1.f, 1.f, 1.f, 1.f), sh0 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 sc1 = sc0, sh1 = sh0;
  if constexpr (PRO) {
    const int ch = (sb.x % a.spj_a) * kSlab + 8 * w + 4 * h;
    sc0 = *(const float4*)(a.pro_scale + ch);
    sh0 = *(const float4*)(a.pro_shift + ch);
    sc1 = *(const float4*)(a.pro_scale + ch + 32);
    sh1 = *(const float4*)(a.pro_shift + ch + 32);
  }
  BnBackCoef cf0{}, cf1{};
  if constexpr (DBB) {
    const int ch = (sb.y % a.spj_d) * kSlab + 8 * w + 4 * h;
    cf0 = load_bnback_coef(a.d_scale, a.d_shift, a.d_c123, a.d_F, ch);
    cf1 = load_bnback_coef(a.d_scale, a.d_shift, a.d_c123, a.d_F, ch + 32);
  }
  const float4* A4 = (const float4*)a.A;
  const float4* D4 = (const float4*)a.D;
  const float4* Z4 = (const float4*)a.d_z;
  const int S_a = a.S_a, S_d = a.S_d;
  const int c40 = t, c41 = t + 256;  // chunk-local float4 index of j even / odd
  float4 ra0, ra1, ra2, ra3, rd0, rd1, rd2, rd3, rz0, rz1, rz2, rz3;
  // float4 index of (row tile, chunk-local index) in a tiled operand with S slabs at slab sl
#define DW_IX(RT, S, SL, C4) (((size_t)(RT) * (S) + (SL)) * 512 + (C4))
#define DW_GLOAD(BASE)                                                            \
  {                                                                               \
    const int t0_ = min((BASE) / kRT, last_rt), t1_ = min((BASE) / kRT + 1, last_rt); \
    ra0 = A4[DW_IX(t0_, S_a, sb.x, c40)];                                         \
    ra1 = A4[DW_IX(t0_, S_a, sb.x, c41)];                                         \
    ra2 = A4[DW_IX(t1_, S_a, sb.x, c40)];                                         \
    ra3 = A4[DW_IX(t1_, S_a, sb.x, c41)];                                         \
    rd0 = D4[DW_IX(t0_, S_d, sb.y, c40)];                                         \
    rd1 = D4[DW_IX(t0_, S_d, sb.y, c41)];                                         \
    rd2 = D4[DW_IX(t1_, S_d, sb.y, c40)];                                         \
    rd3 = D4[DW_IX(t1_, S_d, sb.y, c41)];                                         \
    if constexpr (DBB) {                                                          \
      rz0 = Z4[DW_IX(t0_, S_d, sb.y, c40)];                                       \
      rz1 = Z4[DW_IX(t0_, S_d, sb.y, c41)];                                       \
      rz2 = Z4[DW_IX(t1_, S_d, sb.y, c40)];                                       \
      rz3 = Z4[DW_IX(t1_, S_d, sb.y, c41)];                                       \
    }                                                                             \
  }
  if (r0 < r1) DW_GLOAD(r0);
  for (int base = r0; base < r1; base += 64) {
    __syncthreads();
    const bool v0 = base + lr < r1, v1 = base + 32 + lr < r1;  // row of tile 0 / 1 valid
    if constexpr (PRO) {
      ra0 = bnact4(ra0, sc0, sh0, a.alpha); ra1 = bnact4(ra1, sc1, sh1, a.alpha);
      ra2 = bnact4(ra2, sc0, sh0, a.alpha); ra3 = bnact4(ra3, sc1, sh1, a.alpha);
    }
    if constexpr (DBB) {
      rd0 = bnback4(rd0, rz0, cf0, a.alpha); rd1 = bnback4(rd1, rz1, cf1, a.alpha);
      rd2 = bnback4(rd2, rz2, cf0, a.alpha); rd3 = bnback4(rd3, rz3, cf1, a.alpha);
      if (writer) {
        float4* o = (float4*)a.dz_out;
        const int t0 = base / kRT;
        if (v0) { o[DW_IX(t0, S_d, sb.y, c40)] = rd0; o[DW_IX(t0, S_d, sb.y, c41)] = rd1; }
        if (v1) { o[DW_IX(t0 + 1, S_d, sb.y, c40)] = rd2; o[DW_IX(t0 + 1, S_d, sb.y, c41)] = rd3; }
      }
    }
    {
      // rows past the chunk end contribute nothing (both operands zeroed)
      const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!v0) { ra0 = z4; ra1 = z4; rd0 = z4; rd1 = z4; }
      if (!v1) { ra2 = z4; ra3 = z4; rd2 = z4; rd3 = z4; }
    }
    {
      // transposed scatter: feature 8g + 4h + s -> LDS row, batch row -> column
      const int f0 = 8 * w + 4 * h;  // j even (g = w); j odd adds 32 (g = w + 4)
      float* a0 = As + f0 * kDwLd + lr;
      float* d0 = Ds + f0 * kDwLd + lr;
#define DW_PUT(P, F4, COL)                 \
  P[(COL)] = (F4).x;                       \
  P[(COL) + kDwLd] = (F4).y;               \
  P[(COL) + 2 * kDwLd] = (F4).z;           \
  P[(COL) + 3 * kDwLd] = (F4).w;
      DW_PUT(a0, ra0, 0) DW_PUT(a0, ra1, 32 * kDwLd) DW_PUT(a0, ra2, 32) DW_PUT(a0, ra3, 32 * kDwLd + 32)
      DW_PUT(d0, rd0, 0) DW_PUT(d0, rd1, 32 * kDwLd) DW_PUT(d0, rd2, 32) DW_PUT(d0, rd3, 32 * kDwLd + 32)
#undef DW_PUT
    }
    __syncthreads();
    if (base + 64 < r1) DW_GLOAD(base + 64);
    const float* Ap = As + (32 * wp + lr) * kDwLd + 4 * h;
    const float* Dp = Ds + (32 * wq + lr) * kDwLd + 4 * h;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const float4 av = *(const float4*)(Ap + 8 * g);
      const float4 dv = *(const float4*)(Dp + 8 * g);
      acc = MFMA32(av.x, dv.x, acc);
      acc = MFMA32(av.y, dv.y, acc);
      acc = MFMA32(av.z, dv.z, acc);
      acc = MFMA32(av.w, dv.w, acc);
    }
  }
#undef DW_GLOAD
#undef DW_IX
  float* out = a.part + ((size_t)chunk * a.nblk + b) * 4096;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int p = 32 * wp + (k & 3) + 8 * (k >> 2) + 4 * h;
    out[p * 64 + 32 * wq + lr] = acc[k];
  }
}

void launch_gemm_dw(const GemmDwArgs& a, hipStream_t s) {
  const int grid = a.nblk * a.nchunks;
  const bool pro = a.pro_scale != nullptr, dbb = a.d_bnback != 0;
  if (pro && dbb)
    hipLaunchKernelGGL((gemm_dw_kernel<true, true>), dim3(grid), dim3(256), 0, s, a);
  else if (pro)
    hipLaunchKernelGGL((gemm_dw_kernel<true, false>), dim3(grid), dim3(256), 0, s, a);
  else if (dbb)
    hipLaunchKernelGGL((gemm_dw_kernel<false, true>), dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_dw_kernel<false, false>), dim3(grid), dim3(256), 0, s, a);
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
