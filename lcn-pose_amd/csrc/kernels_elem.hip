// BatchNorm with batch statistics, LeakyReLU, residual and their backward
// (gfx950).  Replaces Keras BatchNormalization(axis=-1) in training mode on
// the [B, 17, F] view (models_att.py:588-612; tf.nn.moments mean / biased
// variance, tf.nn.batch_normalization's x*inv + (beta - mean*inv)),
// tf.nn.leaky_relu(alpha=0.2) and the residual add (models_att.py:704).
//
// Statistics are reduced in three levels: per 128-row group the producing
// GEMM's epilogue writes (sum, sum of squared deviations about the tile mean)
// -- or, backward, (sum du, sum du*zhat) -- as float; colreduce merges the
// tiles of every column in float64; the channel kernels merge the 17 joint
// columns of a channel and finish.  The forward merge uses
//   sum_b (z_b - mu)^2 = sum_t [M2_t + s_t^2 / n_t] - S^2 / N
// in float64: each term is exact to ~1e-16 relative, so the cancellation of
// the last difference costs nothing at float output precision.  With several
// GPUs the channel sums are all-reduced (RCCL, float64) between the phases
// (SyncBN): one all-reduce of 2F doubles per BN layer and direction.
#include <algorithm>
#include "lcn_internal.h"

namespace lcn {

// tf.nn.leaky_relu: max(alpha * u, u)  (alpha < 1)
__device__ __forceinline__ float leaky(float u, float alpha) { return fmaxf(u * alpha, u); }

// Column sums of tile partials part[n_tiles][H] in float64, split over
// kColSplit tile groups (grid.y) so the reduction fills the chip:
// out[p][col] = sum over tiles t of group p (t = 4p + w mod 4P, waves w) of
//   mode 0: (x, y)          mode 1: (x, y + x^2 / n_t)
// fixed-order combines throughout (deterministic).  The finish kernels add
// the kColSplit groups.
// publish = true: the sums are written through to memory (sc1 stores), for the
// fused kernels below whose last workgroup reads every workgroup's sums
template <bool kPublish>
__device__ __forceinline__ void colreduce_body(const float2* __restrict__ part, int n_tiles,
                                               int tile_rows, int B, int H, int mode,
                                               double2* __restrict__ out) {
  __shared__ double2 red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane, p = blockIdx.y, P = gridDim.y;
  double a = 0.0, b = 0.0;
  if (col < H) {
    for (int t = 4 * p + w; t < n_tiles; t += 4 * P) {
      const float2 v = part[(size_t)t * H + col];
      a += (double)v.x;
      if (mode == 1) {
        const double nt = (double)min(tile_rows, B - t * tile_rows);
        b += (double)v.y + (double)v.x * (double)v.x / nt;
      } else {
        b += (double)v.y;
      }
    }
  }
  red[w][lane] = make_double2(a, b);
  __syncthreads();
  if (w == 0 && col < H) {
    const double sx = (red[0][lane].x + red[1][lane].x) + (red[2][lane].x + red[3][lane].x);
    const double sy = (red[0][lane].y + red[1][lane].y) + (red[2][lane].y + red[3][lane].y);
    double2* o = out + (size_t)p * H + col;
    if constexpr (kPublish) {
      __hip_atomic_store(&o->x, sx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&o->y, sy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      *o = make_double2(sx, sy);
    }
  }
}

__global__ __launch_bounds__(256) void colreduce_kernel(const float2* __restrict__ part,
                                                        int n_tiles, int tile_rows, int B, int H,
                                                        int mode, double2* __restrict__ out) {
  colreduce_body<false>(part, n_tiles, tile_rows, B, H, mode, out);
}

// The column reduce and the BN finish in ONE launch: every workgroup publishes
// its sums (write-through stores, drained by the storing wave) and draws a
// ticket; the workgroup that draws the last one acquires (its CU's L1 is
// invalidated) and runs the
// finish that used to be a launch of its own (plain loads after the acquire and
// a workgroup barrier).  One relaxed device-scope atomic
// per workgroup, one acquire in the last workgroup only -- the form with a
// device-scope fence in EVERY workgroup (release + acquire) measured ~9 us
// slower per launch than the two kernels, because each release writes back an
// XCD's L2, dirty from the GEMM before.  The last workgroup resets the ticket
// for the next launch.  Returns true in the last workgroup (all its threads).
__device__ __forceinline__ bool publish_and_draw(int* ticket, int total) {
  __shared__ int is_last;
  // only wave 0 stored; it drains its stores before its lane 0 draws
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = t == total - 1;
    if (is_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return is_last != 0;
}

void launch_colreduce(const float2* part, int n_tiles, int tile_rows, int B, int H, int mode,
                      double2* out, hipStream_t s) {
  hipLaunchKernelGGL(colreduce_kernel, dim3((H + 63) / 64, kColSplit), dim3(256), 0, s, part,
                     n_tiles, tile_rows, B, H, mode, out);
}

// Both finish kernels run as ONE workgroup of 1024 threads: first the
// kColSplit tile groups of every column are added (fixed order) into LDS,
// then one thread per channel adds its 17 joint columns and finishes.
// kSameLaunch: the sums were published by other workgroups of this launch
// (colreduce_body<true>) and this workgroup has acquired (publish_and_draw): its
// plain loads miss the invalidated L1 and find the written-through sums.  One
// thread per column, the kColSplit loads of a column in flight together.
template <bool kSameLaunch = false>
__device__ __forceinline__ void colsum_groups_lds(const double2* col, int H, double2* cs) {
  for (int c = threadIdx.x; c < H; c += blockDim.x) {
    double2 v[kColSplit];
#pragma unroll
    for (int p = 0; p < kColSplit; ++p) v[p] = col[(size_t)p * H + c];
    double x = 0.0, y = 0.0;
#pragma unroll
    for (int p = 0; p < kColSplit; ++p) {
      x += v[p].x;
      y += v[p].y;
    }
    cs[c] = make_double2(x, y);
  }
  __syncthreads();
}

// The same column sums straight from the GEMM's tile partials part[n_tiles][H]
// (float64, tiles in order; mode as colreduce), for launches of few tiles:
// one kernel instead of colreduce + finish.
__device__ __forceinline__ void colsum_tiles_lds(const float2* __restrict__ part, int n_tiles,
                                                 int tile_rows, int B, int H, int mode, double2* cs) {
  for (int c = threadIdx.x; c < H; c += blockDim.x) {
    double x = 0.0, y = 0.0;
    float2 pv[8];  // n_tiles <= 8: all loads in flight together
#pragma unroll
    for (int t = 0; t < 8; ++t) pv[t] = t < n_tiles ? part[(size_t)t * H + c] : make_float2(0.f, 0.f);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (t >= n_tiles) break;
      const float2 v = pv[t];
      x += (double)v.x;
      if (mode == 1) {
        const double nt = (double)min(tile_rows, B - t * tile_rows);
        y += (double)v.y + (double)v.x * (double)v.x / nt;
      } else {
        y += (double)v.y;
      }
    }
    cs[c] = make_double2(x, y);
  }
  __syncthreads();
}

// Where the finish kernels take their column sums from: colreduce's tile-group
// sums (part == null) or the tile partials themselves.
struct ColSrc {
  const double2* col;
  const float2* part; int n_tiles, tile_rows, B;
};

// Forward BN finish per channel.  Phase 0: complete; 1: local channel sums ->
// acc[2F] (and stop); 2: finish from the all-reduced acc.  zsum (when given)
// receives the per-column sums of z (bias-gradient term of the backward).
struct BnFwdArgs {
  ColSrc src; int H, F, phase; double rows; const RowInfo* ri;
  const float* gamma; const float* beta; float eps; double* acc; BnStats st; double* zsum;
  BnRider rider;
};
template <bool kSameLaunch>
__device__ __forceinline__ void bn_fwd_finish(const BnFwdArgs& a, double2* cs) {
  const ColSrc src = a.src;
  const int H = a.H, F = a.F, phase = a.phase;
  const double rows = a.rows;
  const RowInfo* ri = a.ri;
  const float* gamma = a.gamma;
  const float* beta = a.beta;
  const float eps = a.eps;
  double* acc = a.acc;
  const BnStats st = a.st;
  double* zsum = a.zsum;
  const BnRider rider = a.rider;
  __shared__ double rows_sh;
  if (phase <= 1) {
    if (src.part) colsum_tiles_lds(src.part, src.n_tiles, src.tile_rows, src.B, H, 1, cs);
    else colsum_groups_lds<kSameLaunch>(src.col, H, cs);
  }
  const int J = H / F;
  double rows_global = rows;
  if (rider.kind == kRideRows) {
    if (phase == 1) {  // this rank's slot of the one-hot row vector
      for (int r = threadIdx.x; r < rider.world; r += blockDim.x)
        acc[2 * F + r] = r == rider.rank ? rider.b_local : 0.0;
    } else if (phase == 2) {  // every rank's rows -> this rank's RowInfo
      if (threadIdx.x == 0) {
        double total = 0.0, below = 0.0;
        for (int r = 0; r < rider.world; ++r) {
          const double v = acc[2 * F + r];
          if (r < rider.rank) below += v;
          total += v;
        }
        rider.ri_out->rows_global = total;
        rider.ri_out->row0 = (int64_t)below;
        rows_sh = total;
      }
      __syncthreads();
      rows_global = rows_sh;
    }
  } else if (ri) {
    rows_global = ri->rows_global;
  }
  const double count = rows_global * (double)J;
  for (int ch = threadIdx.x; ch < F; ch += blockDim.x) {
    double S = 0.0, Q = 0.0;
    if (phase <= 1) {
      for (int j = 0; j < J; ++j) {
        const double2 c = cs[j * F + ch];
        S += c.x;
        Q += c.y;
        if (zsum) zsum[j * F + ch] = c.x;
      }
      if (phase == 1) { acc[ch] = S; acc[F + ch] = Q; continue; }
    } else {
      S = acc[ch];
      Q = acc[F + ch];
    }
    const double mu = S / count;
    const double var = fmax(0.0, Q / count - mu * mu);
    const float mean = (float)mu;
    const float rstd = 1.0f / sqrtf((float)var + eps);  // rsqrt(variance + epsilon)
    const float inv = rstd * gamma[ch];                  // inv *= scale
    st.mean[ch] = mean;
    st.rstd[ch] = rstd;
    st.scale[ch] = inv;
    st.shift[ch] = beta[ch] - mean * inv;                // offset - mean * inv
  }
}

__global__ __launch_bounds__(1024) void bn_fwd_finalize_kernel(BnFwdArgs a) {
  extern __shared__ double2 cs[];  // [H]
  bn_fwd_finish<false>(a, cs);
}
// colreduce (mode 1) + forward BN finish (phase 0 or 1) in one launch
__global__ __launch_bounds__(256) void colreduce_bn_fwd_kernel(const float2* __restrict__ part,
                                                               int n_tiles, int tile_rows, int B,
                                                               double2* col, int* ticket,
                                                               BnFwdArgs a) {
  extern __shared__ double2 cs[];  // [H]
  colreduce_body<true>(part, n_tiles, tile_rows, B, a.H, 1, col);
  if (!publish_and_draw(ticket, gridDim.x * gridDim.y)) return;
  bn_fwd_finish<true>(a, cs);
}

void launch_bn_fwd_finalize(const double2* col, const TilePartials& tp, int H, int F, int phase,
                            double rows, const RowInfo* ri, const float* gamma, const float* beta,
                            float eps, double* acc, BnStats st, double* zsum, const BnRider& rider,
                            hipStream_t s) {
  const ColSrc src{col, tp.part, tp.n_tiles, tp.tile_rows, tp.B};
  const BnFwdArgs a{src, H, F, phase, rows, ri, gamma, beta, eps, acc, st, zsum, rider};
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3(1), dim3(1024), H * sizeof(double2), s, a);
}

void launch_colreduce_bn_fwd(const float2* part, int n_tiles, int tile_rows, int B, double2* col,
                             int* ticket, int H, int F, int phase, double rows, const RowInfo* ri,
                             const float* gamma, const float* beta, float eps, double* acc, BnStats st,
                             double* zsum, const BnRider& rider, hipStream_t s) {
  const ColSrc src{col, nullptr, 0, 0, 0};
  const BnFwdArgs a{src, H, F, phase, rows, ri, gamma, beta, eps, acc, st, zsum, rider};
  hipLaunchKernelGGL(colreduce_bn_fwd_kernel, dim3((H + 63) / 64, kColSplit), dim3(256),
                     H * sizeof(double2), s, part, n_tiles, tile_rows, B, col, ticket, a);
}

// Backward BN finish per channel:  dz = c1*du + c2 + c3*z,
//   c1 = gamma*rstd, c3 = -c1*rstd*S2/N, c2 = -c1*S1/N - c3*mean,
//   S1 = sum du = dbeta, S2 = sum du*zhat = dgamma.
// The bias gradient of the layer is sum_b dz per column:
//   db[col] = c1 * sum du[col] + B_local * c2 + c3 * sum z[col].
// dgamma / dbeta / db are the LOCAL contributions (the raw-gradient vector is
// all-reduced later); c123 uses the global sums.  bn = 0 (no BatchNorm):
// dz = du and only db is written.  Phases as bn_fwd_finalize.
struct BnBwdArgs {
  ColSrc src; int H, F, phase, bn; double rows; const RowInfo* ri; double b_local;
  const float* gamma; const float* mean; const float* rstd; double* acc;
  float* dgamma; float* dbeta; float* c123; const double* zsum; float* db;
  BnRider rider;
};
template <bool kSameLaunch>
__device__ __forceinline__ void bn_bwd_finish(const BnBwdArgs& a, double2* cs) {
  const ColSrc src = a.src;
  const int H = a.H, F = a.F, phase = a.phase, bn = a.bn;
  const double rows = a.rows, b_local = a.b_local;
  const RowInfo* ri = a.ri;
  const float* gamma = a.gamma;
  const float* mean = a.mean;
  const float* rstd = a.rstd;
  double* acc = a.acc;
  float* dgamma = a.dgamma;
  float* dbeta = a.dbeta;
  float* c123 = a.c123;
  const double* zsum = a.zsum;
  float* db = a.db;
  const BnRider rider = a.rider;
  if (rider.kind == kRideLoss && threadIdx.x == 0) {
    if (phase == 1) acc[2 * F] = *rider.loss;
    else if (phase == 2) *rider.loss = acc[2 * F];
  }
  if (src.part) colsum_tiles_lds(src.part, src.n_tiles, src.tile_rows, src.B, H, 0, cs);
  else colsum_groups_lds<kSameLaunch>(src.col, H, cs);
  const int J = H / F;
  const double count = (ri ? ri->rows_global : rows) * (double)J;
  for (int ch = threadIdx.x; ch < F; ch += blockDim.x) {
    if (!bn) {
      for (int j = 0; j < J; ++j) db[j * F + ch] = (float)cs[j * F + ch].x;
      continue;
    }
    double S1 = 0.0, S2 = 0.0;
    if (phase <= 1) {
      for (int j = 0; j < J; ++j) {
        const double2 c = cs[j * F + ch];
        S1 += c.x;
        S2 += c.y;
      }
      dgamma[ch] = (float)S2;
      dbeta[ch] = (float)S1;
      if (phase == 1) { acc[ch] = S1; acc[F + ch] = S2; continue; }
    } else {
      S1 = acc[ch];
      S2 = acc[F + ch];
    }
    const double rs = rstd[ch];
    const double c1 = (double)gamma[ch] * rs;
    const double c3 = -c1 * rs * S2 / count;
    const double c2 = -c1 * S1 / count - c3 * (double)mean[ch];
    c123[ch] = (float)c1;
    c123[F + ch] = (float)c2;
    c123[2 * F + ch] = (float)c3;
    for (int j = 0; j < J; ++j) {
      const int cj = j * F + ch;
      db[cj] = (float)(c1 * cs[cj].x + b_local * c2 + c3 * zsum[cj]);
    }
  }
}

__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(BnBwdArgs a) {
  extern __shared__ double2 cs[];  // [H]
  bn_bwd_finish<false>(a, cs);
}
// colreduce (mode 0) + backward BN finish (phase 0 or 1) in one launch
__global__ __launch_bounds__(256) void colreduce_bn_bwd_kernel(const float2* __restrict__ part,
                                                               int n_tiles, int tile_rows, int B,
                                                               double2* col, int* ticket,
                                                               BnBwdArgs a) {
  extern __shared__ double2 cs[];  // [H]
  colreduce_body<true>(part, n_tiles, tile_rows, B, a.H, 0, col);
  if (!publish_and_draw(ticket, gridDim.x * gridDim.y)) return;
  bn_bwd_finish<true>(a, cs);
}

void launch_bn_bwd_finalize(const double2* col, const TilePartials& tp, int H, int F, int phase,
                            int bn, double rows, const RowInfo* ri, double b_local,
                            const float* gamma, const float* mean, const float* rstd, double* acc,
                            float* dgamma, float* dbeta, float* c123, const double* zsum, float* db,
                            const BnRider& rider, hipStream_t s) {
  const ColSrc src{col, tp.part, tp.n_tiles, tp.tile_rows, tp.B};
  const BnBwdArgs a{src, H, F, phase, bn, rows, ri, b_local, gamma, mean, rstd, acc, dgamma, dbeta,
                    c123, zsum, db, rider};
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(1), dim3(1024), H * sizeof(double2), s, a);
}

void launch_colreduce_bn_bwd(const float2* part, int n_tiles, int tile_rows, int B, double2* col,
                             int* ticket, int H, int F, int phase, int bn, double rows,
                             const RowInfo* ri, double b_local, const float* gamma, const float* mean,
                             const float* rstd, double* acc, float* dgamma, float* dbeta, float* c123,
                             const double* zsum, float* db, const BnRider& rider, hipStream_t s) {
  const ColSrc src{col, nullptr, 0, 0, 0};
  const BnBwdArgs a{src, H, F, phase, bn, rows, ri, b_local, gamma, mean, rstd, acc, dgamma, dbeta,
                    c123, zsum, db, rider};
  hipLaunchKernelGGL(colreduce_bn_bwd_kernel, dim3((H + 63) / 64, kColSplit), dim3(256),
                     H * sizeof(double2), s, part, n_tiles, tile_rows, B, col, ticket, a);
}

// h = [res +] leaky(scale*z + shift) over row-tiled [B][S*64] buffers; the
// channel of float4 i is ((i >> 9) % S % (F/64))*64 + 8*g + 4*h with g, h
// from the chunk-local index (lcn_internal.h)
__global__ __launch_bounds__(256) void bn_act_kernel(const float4* __restrict__ z,
                                                     const float4* __restrict__ res,
                                                     float4* __restrict__ h,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ shift, int F, int S,
                                                     float alpha, int64_t n4, Dropout drop_in) {
  const int spj = F / 64;
  const Dropout drop = drop_resolve(drop_in);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(i & 511);
    const int ch = (int)((i >> 9) % S % spj) * 64 + 8 * (c4 >> 6) + 4 * ((c4 >> 5) & 1);
    const float4 sc = *(const float4*)(scale + ch), sh = *(const float4*)(shift + ch);
    float4 v = z[i];
    v.x = leaky(fmaf(v.x, sc.x, sh.x), alpha);
    v.y = leaky(fmaf(v.y, sc.y, sh.y), alpha);
    v.z = leaky(fmaf(v.z, sc.z, sh.z), alpha);
    v.w = leaky(fmaf(v.w, sc.w, sh.w), alpha);
    if (drop.rate > 0.f) {  // row / column of this float4 in the row-tile layout
      const int64_t row = (i >> 9) / S * kRT + (c4 & 31);
      const int col = (int)((i >> 9) % S) * 64 + 8 * (c4 >> 6) + 4 * ((c4 >> 5) & 1);
      v.x = drop_apply(drop, row, col, v.x);
      v.y = drop_apply(drop, row, col + 1, v.y);
      v.z = drop_apply(drop, row, col + 2, v.z);
      v.w = drop_apply(drop, row, col + 3, v.w);
    }
    if (res) {
      const float4 r = res[i];
      v.x = r.x + v.x; v.y = r.y + v.y; v.z = r.z + v.z; v.w = r.w + v.w;
    }
    h[i] = v;
  }
}

void launch_bn_act(const float* z, const float* res, float* h, const float* scale,
                   const float* shift, int F, float alpha, int B, int S, const Dropout& drop,
                   hipStream_t s) {
  const int64_t n4 = tiled_floats(B, S) / 4;
  const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(bn_act_kernel, dim3(grid), dim3(256), 0, s, (const float4*)z,
                     (const float4*)res, (float4*)h, scale, shift, F, S, alpha, n4, drop);
}

// The ranks' batch rows of a step: begin fills this rank's slot (the others
// zero), an all-reduce (sum) gathers them, finish derives this rank's RowInfo.
__global__ void rows_begin_kernel(double* rows, int world, int rank, double B) {
  const int r = threadIdx.x;
  if (r < world) rows[r] = r == rank ? B : 0.0;
}
__global__ void rows_finish_kernel(const double* rows, int world, int rank, RowInfo* ri) {
  if (threadIdx.x != 0) return;
  double total = 0.0, below = 0.0;
  for (int r = 0; r < world; ++r) {
    if (r < rank) below += rows[r];
    total += rows[r];
  }
  ri->rows_global = total;
  ri->row0 = (int64_t)below;
}
void launch_rows_begin(double* rows, int world, int rank, int64_t B, hipStream_t s) {
  hipLaunchKernelGGL(rows_begin_kernel, dim3(1), dim3(256), 0, s, rows, world, rank, (double)B);
}
void launch_rows_finish(const double* rows, int world, int rank, RowInfo* ri, hipStream_t s) {
  hipLaunchKernelGGL(rows_finish_kernel, dim3(1), dim3(64), 0, s, rows, world, rank, ri);
}

}  // namespace lcn
