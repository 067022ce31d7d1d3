// The two thin layers at the ends of the LCN (gfx950, VALU fp32):
//   lift   z0 = x . W1e + b1        (models_att.py:714-729), K = 17*in_F
//   output y  = h . W4e + b4, out = [x_xy + y_xy, y_z], MSE loss and dy
//                                   (models_att.py:749-773, :356)
// and their gradients.  Both are HBM-bound: each reads or writes one
// [B, J*F] activation once; the weights live in registers / LDS.
#include "lcn_internal.h"

namespace lcn {

// out[b, s*64+f] = bias + sum_{u in umask[s], c < C} small[b, u*C+c] * coef[s][u][c][f]
// One workgroup = 64 rows x one 64-feature slab; lane = feature; 4 waves x 16 rows.
template <int C>
__global__ __launch_bounds__(256) void expand_kernel(ExpandArgs a) {
  __shared__ float sm[64 * 52];
  __shared__ float red[2][4][64];
  const int rt = blockIdx.x / a.n_slabs, s = blockIdx.x - rt * a.n_slabs;
  const int row0 = rt * 64;
  const int t = threadIdx.x, f = t & 63, w = t >> 6;
  constexpr int JC = kJ * C;
  for (int i = t; i < 64 * JC; i += 256) {
    const int r = i / JC, c = i - r * JC;
    sm[r * 52 + c] = (row0 + r < a.B) ? a.small[(size_t)(row0 + r) * a.lds_small + c] : 0.f;
  }
  const unsigned m = a.umask[s];
  float cf[kJ][C];
#pragma unroll
  for (int u = 0; u < kJ; ++u)
#pragma unroll
    for (int c = 0; c < C; ++c)
      cf[u][c] = ((m >> u) & 1u) ? a.coef[((size_t)(s * kJ + u) * C + c) * 64 + f] : 0.f;
  const float bias = a.bias ? a.bias[s * 64 + f] : 0.f;
  __syncthreads();
  float v[16];
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int r = w + 4 * k;
    const float* srow = sm + r * 52;
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < kJ; ++u) {
      if ((m >> u) & 1u) {
#pragma unroll
        for (int c = 0; c < C; ++c) acc = fmaf(srow[u * C + c], cf[u][c], acc);
      }
    }
    acc += bias;
    v[k] = acc;
    if (row0 + r < a.B) {
      a.out[(size_t)(row0 + r) * a.ldo + s * 64 + f] = acc;
      sum += acc;
    }
  }
  if (a.stat == nullptr) return;
  const int nval = min(64, a.B - row0);
  red[0][w][f] = sum;
  __syncthreads();
  const float tot = (red[0][0][f] + red[0][1][f]) + (red[0][2][f] + red[0][3][f]);
  const float mean = tot / (float)nval;
  float m2 = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (row0 + w + 4 * k < a.B) {
      const float d = v[k] - mean;
      m2 = fmaf(d, d, m2);
    }
  }
  red[1][w][f] = m2;
  __syncthreads();
  if (w == 0) {
    const float q = (red[1][0][f] + red[1][1][f]) + (red[1][2][f] + red[1][3][f]);
    a.stat[(size_t)rt * a.ldo + s * 64 + f] = make_float2(tot, q);
  }
}

void launch_expand(const ExpandArgs& a, hipStream_t s) {
  const int grid = ((a.B + 63) / 64) * a.n_slabs;
  if (a.C == 2) hipLaunchKernelGGL(expand_kernel<2>, dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(expand_kernel<3>, dim3(grid), dim3(256), 0, s, a);
}

// part[chunk][s][u*C+c][f] = sum_{b in chunk} big[b, s*64+f] * small[b, u*C+c]
template <int C>
__global__ __launch_bounds__(256) void outer_kernel(OuterArgs a) {
  constexpr int JC = kJ * C;
  __shared__ float sm[64 * 52];
  const int chunk = blockIdx.x / a.n_slabs, s = blockIdx.x - chunk * a.n_slabs;
  const int t = threadIdx.x, f = t & 63, w = t >> 6;
  const int r0 = chunk * a.chunk_rows, r1 = min(a.B, r0 + a.chunk_rows);
  const unsigned m = a.umask[s];
  float acc[kJ][C];
#pragma unroll
  for (int u = 0; u < kJ; ++u)
#pragma unroll
    for (int c = 0; c < C; ++c) acc[u][c] = 0.f;
  const float* bsrc = a.big + s * 64 + f;
  for (int base = r0; base < r1; base += 64) {
    __syncthreads();
    for (int i = t; i < 64 * JC; i += 256) {
      const int r = i / JC, c = i - r * JC;
      sm[r * 52 + c] = (base + r < r1) ? a.small[(size_t)(base + r) * a.lds_small + c] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
      const int r = w + 4 * k;
      const float bv = (base + r < r1) ? bsrc[(size_t)(base + r) * a.ldb] : 0.f;
      const float* srow = sm + r * 52;
#pragma unroll
      for (int u = 0; u < kJ; ++u) {
        if ((m >> u) & 1u) {
#pragma unroll
          for (int c = 0; c < C; ++c) acc[u][c] = fmaf(bv, srow[u * C + c], acc[u][c]);
        }
      }
    }
  }
  // reduce the 4 waves through sm (17*C*64 <= 64*52 floats): waves 1..3 publish,
  // wave 0 sums in fixed order
  float* out = a.part + ((size_t)chunk * a.n_slabs + s) * JC * 64;
  for (int src = 1; src < 4; ++src) {
    __syncthreads();
    if (w == src) {
#pragma unroll
      for (int u = 0; u < kJ; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c) sm[(u * C + c) * 64 + f] = acc[u][c];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int u = 0; u < kJ; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c) acc[u][c] += sm[(u * C + c) * 64 + f];
    }
  }
  if (w == 0) {
#pragma unroll
    for (int u = 0; u < kJ; ++u)
#pragma unroll
      for (int c = 0; c < C; ++c) out[(u * C + c) * 64 + f] = acc[u][c];
  }
}

void launch_outer(const OuterArgs& a, hipStream_t s) {
  const int grid = a.nchunks * a.n_slabs;
  if (a.C == 2) hipLaunchKernelGGL(outer_kernel<2>, dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(outer_kernel<3>, dim3(grid), dim3(256), 0, s, a);
}

__global__ void outer_reduce_kernel(const float* __restrict__ part, int nchunks, int n_slabs, int C,
                                    int mode, float* __restrict__ dW) {
  const int JC = kJ * C;
  const int total = n_slabs * JC * 64;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  float s = 0.f;
  for (int c = 0; c < nchunks; ++c) s += part[(size_t)c * total + e];
  const int f = e & 63, uc = (e >> 6) % JC, sl = (e >> 6) / JC;
  if (mode == 0) dW[(size_t)uc * (n_slabs * 64) + sl * 64 + f] = s;
  else dW[(size_t)(sl * 64 + f) * JC + uc] = s;
}

void launch_outer_reduce(const float* part, int nchunks, int n_slabs, int C, int mode, float* dW,
                         hipStream_t s) {
  const int total = n_slabs * kJ * C * 64;
  hipLaunchKernelGGL(outer_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, s, part,
                     nchunks, n_slabs, C, mode, dW);
}

// Output layer.  One workgroup = 64 rows; thread = (row r, joint group grp)
// with joints grp, grp+4, ... (<= 5 joints x 3 coordinates in registers).
// Per input slab the 64x64 activation tile and the 64x51 weight rows are
// staged in LDS; the weight reads are wave-uniform broadcasts.
__global__ __launch_bounds__(256) void out_fwd_kernel(OutFwdArgs a) {
  __shared__ float Hs[64 * 65];
  __shared__ float Ws[64 * 52];
  __shared__ double lred[256];
  const int row0 = blockIdx.x * 64;
  const int t = threadIdx.x, r = t & 63, grp = t >> 6;
  float acc[5][3];
#pragma unroll
  for (int m = 0; m < 5; ++m)
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[m][c] = 0.f;
  const int fc = t & 15, rr = t >> 4;
  for (int si = 0; si < a.n_in_slabs; ++si) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = rr + 16 * q;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row0 + row < a.B) v = *(const float4*)(a.h + (size_t)(row0 + row) * a.ldh + si * 64 + 4 * fc);
      float* d = Hs + row * 65 + 4 * fc;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
    for (int i = t; i < 64 * 51; i += 256) {
      const int p = i / 51, c = i - p * 51;
      Ws[p * 52 + c] = a.w4[(size_t)(si * 64 + p) * 51 + c];
    }
    __syncthreads();
    const float* hrow = Hs + r * 65;
#pragma unroll 4
    for (int p = 0; p < 64; ++p) {
      const float hv = hrow[p];
      const float* wrow = Ws + p * 52;
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        const int j = grp + 4 * m;
        if (j < kJ) {
#pragma unroll
          for (int c = 0; c < 3; ++c) acc[m][c] = fmaf(hv, wrow[3 * j + c], acc[m][c]);
        }
      }
    }
  }
  const int row = row0 + r;
  double lsum = 0.0;
  if (row < a.B) {
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const int j = grp + 4 * m;
      if (j < kJ) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float y = acc[m][c] + a.b4[3 * j + c];
          const float o = c < 2 ? a.x[(size_t)row * (kJ * a.in_f) + a.in_f * j + c] + y : y;
          a.out[(size_t)row * 51 + 3 * j + c] = o;
          if (a.lab) {
            const float d = o - a.lab[(size_t)row * 51 + 3 * j + c];
            lsum += (double)d * (double)d;
            if (a.dy) a.dy[(size_t)row * 51 + 3 * j + c] = a.dscale * d;
          }
        }
      }
    }
  }
  if (a.loss_part) {
    lred[t] = lsum;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if (t < st) lred[t] += lred[t + st];
      __syncthreads();
    }
    if (t == 0) a.loss_part[blockIdx.x] = lred[0];
  }
}

void launch_out_fwd(const OutFwdArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(out_fwd_kernel, dim3((a.B + 63) / 64), dim3(256), 0, s, a);
}

__global__ void loss_finalize_kernel(const double* part, int n, double* out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

void launch_loss_finalize(const double* part, int n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, part, n, out);
}

}  // namespace lcn
