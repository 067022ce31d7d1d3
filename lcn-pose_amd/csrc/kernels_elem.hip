// BatchNorm with batch statistics, LeakyReLU, residual and their backward
// (gfx950).  Replaces Keras BatchNormalization(axis=-1) in training mode on
// the [B, 17, F] view (models_att.py:588-612; tf.nn.moments two-pass mean /
// biased variance, tf.nn.batch_normalization's x*inv + (beta - mean*inv)),
// tf.nn.leaky_relu(alpha=0.2) and the residual add (models_att.py:704).
//
// Statistics are reduced in two levels: per-tile (sum, sum of squared
// deviations about the tile mean) written by the producing kernel's
// epilogue, then merged here in float64 (exact decomposition, no E[z^2]-mu^2
// cancellation).  With several GPUs the merge is split into phases around an
// RCCL all-reduce of the float64 partial sums (SyncBN).
#include <algorithm>
#include "lcn_internal.h"

namespace lcn {

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  // 256 threads
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// One workgroup per channel ch; entries (tile t, joint-slab j) at column j*F + ch.
__global__ __launch_bounds__(256) void bn_finalize_kernel(
    const float2* __restrict__ part, int n_tiles, int tile_rows, int B, int H, int F,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, double count,
    double* acc1, double* acc2, int phase, BnStats st) {
  __shared__ double red[4];
  const int ch = blockIdx.x;
  const int J = H / F;
  const int n = n_tiles * J;
  double mu = 0.0, s2 = 0.0;
  if (phase == 0 || phase == 1) {
    double s1 = 0.0;
    for (int e = threadIdx.x; e < n; e += 256) {
      const int t = e / J, j = e - t * J;
      s1 += (double)part[(size_t)t * H + j * F + ch].x;
    }
    s1 = block_sum_d(s1, red);
    if (phase == 1) {
      if (threadIdx.x == 0) acc1[ch] = s1;
      return;
    }
    mu = s1 / count;
  }
  if (phase == 2) mu = acc1[ch] / count;
  if (phase == 0 || phase == 2) {
    double q = 0.0;
    for (int e = threadIdx.x; e < n; e += 256) {
      const int t = e / J, j = e - t * J;
      const float2 p = part[(size_t)t * H + j * F + ch];
      const double nt = (double)min(tile_rows, B - t * tile_rows);
      const double d = (double)p.x / nt - mu;
      q += (double)p.y + nt * d * d;
    }
    s2 = block_sum_d(q, red);
    if (phase == 2) {
      if (threadIdx.x == 0) acc2[ch] = s2;
      return;
    }
  }
  if (phase == 3) { mu = acc1[ch] / count; s2 = acc2[ch]; }
  if (threadIdx.x == 0) {
    const float mean = (float)mu;
    const float var = (float)(s2 / count);
    const float rstd = 1.0f / sqrtf(var + eps);   // rsqrt(variance + epsilon)
    const float inv = rstd * gamma[ch];           // inv *= scale
    st.mean[ch] = mean;
    st.rstd[ch] = rstd;
    st.scale[ch] = inv;
    st.shift[ch] = beta[ch] - mean * inv;         // offset - mean * inv
  }
}

void launch_bn_finalize(const float2* part, int n_row_tiles, int tile_rows, int B, int H, int F,
                        const float* gamma, const float* beta, float eps, double count,
                        double* acc1, double* acc2, int phase, BnStats st, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(F), dim3(256), 0, s, part, n_row_tiles, tile_rows, B,
                     H, F, gamma, beta, eps, count, acc1, acc2, phase, st);
}

__device__ __forceinline__ float leaky(float u, float alpha) { return u > 0.f ? u : u * alpha; }

__global__ __launch_bounds__(256) void bn_act_kernel(const float4* __restrict__ z,
                                                     const float4* __restrict__ res,
                                                     float4* __restrict__ h,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ shift, int F,
                                                     float alpha, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int ch = (int)((i * 4) % F);
    const float4 sc = *(const float4*)(scale + ch), sh = *(const float4*)(shift + ch);
    float4 v = z[i];
    v.x = leaky(fmaf(v.x, sc.x, sh.x), alpha);
    v.y = leaky(fmaf(v.y, sc.y, sh.y), alpha);
    v.z = leaky(fmaf(v.z, sc.z, sh.z), alpha);
    v.w = leaky(fmaf(v.w, sc.w, sh.w), alpha);
    if (res) {
      const float4 r = res[i];
      v.x = r.x + v.x; v.y = r.y + v.y; v.z = r.z + v.z; v.w = r.w + v.w;
    }
    h[i] = v;
  }
}

void launch_bn_act(const float* z, const float* res, float* h, const float* scale,
                   const float* shift, int F, float alpha, int B, int H, hipStream_t s) {
  const int64_t n4 = (int64_t)B * H / 4;
  const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(bn_act_kernel, dim3(grid), dim3(256), 0, s, (const float4*)z,
                     (const float4*)res, (float4*)h, scale, shift, F, alpha, n4);
}

// One workgroup = kEwRows rows x one 64-column slab; lane = column.
__global__ __launch_bounds__(256) void bnback_reduce_kernel(
    const float* __restrict__ dh, const float* __restrict__ z, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ mean, const float* __restrict__ rstd,
    int F, float alpha, int B, int H, float2* __restrict__ part) {
  __shared__ float red[2][4][64];
  const int nsl = H / 64;
  const int rt = blockIdx.x / nsl, sl = blockIdx.x - rt * nsl;
  const int t = threadIdx.x, f = t & 63, w = t >> 6;
  const int col = sl * 64 + f, ch = col % F;
  const float sc = scale[ch], sh = shift[ch], mu = mean[ch], rs = rstd[ch];
  const int r0 = rt * kEwRows, r1 = min(B, r0 + kEwRows);
  float s1 = 0.f, s2 = 0.f;
  for (int r = r0 + w; r < r1; r += 4) {
    const size_t o = (size_t)r * H + col;
    const float zv = z[o], g = dh[o];
    const float u = fmaf(zv, sc, sh);
    const float du = u > 0.f ? g : g * alpha;
    s1 += du;
    s2 = fmaf(du, (zv - mu) * rs, s2);
  }
  red[0][w][f] = s1;
  red[1][w][f] = s2;
  __syncthreads();
  if (w == 0) {
    part[(size_t)rt * H + col] =
        make_float2((red[0][0][f] + red[0][1][f]) + (red[0][2][f] + red[0][3][f]),
                    (red[1][0][f] + red[1][1][f]) + (red[1][2][f] + red[1][3][f]));
  }
}

void launch_bnback_reduce(const float* dh, const float* z, const float* scale, const float* shift,
                          const float* mean, const float* rstd, int F, float alpha, int batch_norm,
                          int B, int H, float2* part, hipStream_t s) {
  (void)batch_norm;
  const int grid = ((B + kEwRows - 1) / kEwRows) * (H / 64);
  hipLaunchKernelGGL(bnback_reduce_kernel, dim3(grid), dim3(256), 0, s, dh, z, scale, shift, mean,
                     rstd, F, alpha, B, H, part);
}

// c123 = [c1 | c2 | c3] (3F):  dz = c1*du + c2 + c3*z, with
//   c1 = gamma*rstd, c3 = -c1*rstd*S2/N, c2 = -c1*S1/N - c3*mean,
//   S1 = sum du = dbeta, S2 = sum du*zhat = dgamma   
__global__ __launch_bounds__(256) void bnback_finalize_kernel(
    const float2* __restrict__ part, int n_tiles, int H, int F, double count,
    const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ rstd,
    double* acc, int phase, float* dgamma, float* dbeta, float* c123) {
  __shared__ double red[4];
  const int ch = blockIdx.x;
  const int J = H / F;
  double S1, S2;
  if (phase == 0 || phase == 1) {
    double a1 = 0.0, a2 = 0.0;
    const int n = n_tiles * J;
    for (int e = threadIdx.x; e < n; e += 256) {
      const int t = e / J, j = e - t * J;
      const float2 p = part[(size_t)t * H + j * F + ch];
      a1 += (double)p.x;
      a2 += (double)p.y;
    }
    S1 = block_sum_d(a1, red);
    S2 = block_sum_d(a2, red);
    if (phase == 1) {
      if (threadIdx.x == 0) { acc[ch] = S1; acc[F + ch] = S2; }
      return;
    }
  } else {
    S1 = acc[ch];
    S2 = acc[F + ch];
  }
  if (threadIdx.x == 0) {
    const double rs = rstd[ch];
    const double c1 = (double)gamma[ch] * rs;
    const double c3 = -c1 * rs * S2 / count;
    const double c2 = -c1 * S1 / count - c3 * (double)mean[ch];
    c123[ch] = (float)c1;
    c123[F + ch] = (float)c2;
    c123[2 * F + ch] = (float)c3;
    dgamma[ch] = (float)S2;
    dbeta[ch] = (float)S1;
  }
}

void launch_bnback_finalize(const float2* part, int n_tiles, int H, int F, double count,
                            const float* gamma, const float* mean, const float* rstd, double* acc,
                            int phase, float* dgamma, float* dbeta, float* c123, hipStream_t s) {
  hipLaunchKernelGGL(bnback_finalize_kernel, dim3(F), dim3(256), 0, s, part, n_tiles, H, F, count,
                     gamma, mean, rstd, acc, phase, dgamma, dbeta, c123);
}

__global__ __launch_bounds__(256) void bnback_apply_kernel(
    const float* __restrict__ dh, const float* __restrict__ z, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ c123, int F, float alpha, int B,
    int H, float* __restrict__ dz, float* __restrict__ bpart) {
  __shared__ float red[4][64];
  const int nsl = H / 64;
  const int rt = blockIdx.x / nsl, sl = blockIdx.x - rt * nsl;
  const int t = threadIdx.x, f = t & 63, w = t >> 6;
  const int col = sl * 64 + f, ch = col % F;
  const float sc = scale[ch], sh = shift[ch];
  const float c1 = c123[ch], c2 = c123[F + ch], c3 = c123[2 * F + ch];
  const int r0 = rt * kEwRows, r1 = min(B, r0 + kEwRows);
  float sb = 0.f;
  for (int r = r0 + w; r < r1; r += 4) {
    const size_t o = (size_t)r * H + col;
    const float zv = z[o], g = dh[o];
    const float u = fmaf(zv, sc, sh);
    const float du = u > 0.f ? g : g * alpha;
    const float d = fmaf(c1, du, fmaf(c3, zv, c2));
    dz[o] = d;
    sb += d;
  }
  red[w][f] = sb;
  __syncthreads();
  if (w == 0) bpart[(size_t)rt * H + col] = (red[0][f] + red[1][f]) + (red[2][f] + red[3][f]);
}

void launch_bnback_apply(const float* dh, const float* z, const float* scale, const float* shift,
                         const float* c123, int F, float alpha, int batch_norm, int B, int H,
                         float* dz, float* bpart, hipStream_t s) {
  (void)batch_norm;
  const int grid = ((B + kEwRows - 1) / kEwRows) * (H / 64);
  hipLaunchKernelGGL(bnback_apply_kernel, dim3(grid), dim3(256), 0, s, dh, z, scale, shift, c123,
                     F, alpha, B, H, dz, bpart);
}

__global__ void colsum_kernel(const float* __restrict__ part, int n_tiles, int H,
                              float* __restrict__ out) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= H) return;
  double s = 0.0;
  for (int t = 0; t < n_tiles; ++t) s += (double)part[(size_t)t * H + col];
  out[col] = (float)s;
}

void launch_colsum(const float* part, int n_tiles, int H, float* out, hipStream_t s) {
  hipLaunchKernelGGL(colsum_kernel, dim3((H + 255) / 256), dim3(256), 0, s, part, n_tiles, H, out);
}

// per-tile column sums of a narrow [B][ncols <= 64] matrix (the output bias gradient)
__global__ __launch_bounds__(256) void colpart_kernel(const float* __restrict__ src, int B,
                                                      int ncols, int ld, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int t = threadIdx.x, c = t & 63, w = t >> 6;
  const int r0 = blockIdx.x * kEwRows, r1 = min(B, r0 + kEwRows);
  float s = 0.f;
  if (c < ncols)
    for (int r = r0 + w; r < r1; r += 4) s += src[(size_t)r * ld + c];
  red[w][c] = s;
  __syncthreads();
  if (w == 0 && c < ncols)
    part[(size_t)blockIdx.x * ncols + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

void launch_colpart(const float* src, int B, int ncols, int ld, float* part, hipStream_t s) {
  hipLaunchKernelGGL(colpart_kernel, dim3((B + kEwRows - 1) / kEwRows), dim3(256), 0, s, src, B,
                     ncols, ld, part);
}

}  // namespace lcn
