// Per-step parameter kernels (gfx950): the learnable LC mask, clip_by_norm,
// mask_weights, weight packing for the block-sparse GEMMs, the mask / clip
// backward and the fused Adam update.
//
//   M = softmax(V, axis=0) (.) 1[N^T != 0]        models_att.py:557-571
//   W_c = W / max(||W||_F, 1)                     tf.clip_by_norm, :659/690/726/762
//   W_e[i,p,j,q] = W_c[i,p,j,q] * M[i,j]          mask_weights, :576-586
//   AdamOptimizer (TF1 ApplyAdam), exp decay      :392-409
#include <algorithm>
#include "lcn_internal.h"

namespace lcn {

__global__ void mask_kernel(const float* __restrict__ V, const float* __restrict__ C, int learnable,
                            float* __restrict__ M, float* __restrict__ S) {
  const int j = threadIdx.x;
  if (j >= kJ) return;
  if (!learnable) {
    for (int i = 0; i < kJ; ++i) { M[i * kJ + j] = C[i * kJ + j]; S[i * kJ + j] = 0.f; }
    return;
  }
  float mx = V[j];
  for (int i = 1; i < kJ; ++i) mx = fmaxf(mx, V[i * kJ + j]);
  float e[kJ];
  float sum = 0.f;
  for (int i = 0; i < kJ; ++i) { e[i] = expf(V[i * kJ + j] - mx); sum += e[i]; }
  for (int i = 0; i < kJ; ++i) {
    const float s = e[i] / sum;
    S[i * kJ + j] = s;
    M[i * kJ + j] = s * (C[i * kJ + j] != 0.f ? 1.f : 0.f);
  }
}

void launch_mask(const float* V, const float* Cmat, int learnable, float* M, float* S, hipStream_t s) {
  hipLaunchKernelGGL(mask_kernel, dim3(1), dim3(64), 0, s, V, Cmat, learnable, M, S);
}

__global__ __launch_bounds__(256) void wnorm_part_kernel(const float* __restrict__ params,
                                                         const int64_t* __restrict__ offs,
                                                         const int64_t* __restrict__ sizes,
                                                         double* __restrict__ part, int ppl) {
  __shared__ double red[4];
  const int l = blockIdx.y, p = blockIdx.x;
  const float* w = params + offs[l];
  const int64_t n = sizes[l];
  // four independent chains per thread: the float64 multiply-adds are
  // latency bound otherwise (fixed order, deterministic)
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  const int64_t stride = (int64_t)ppl * 256;
  int64_t i = (int64_t)p * 256 + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const double v0 = w[i], v1 = w[i + stride], v2 = w[i + 2 * stride], v3 = w[i + 3 * stride];
    s0 += v0 * v0; s1 += v1 * v1; s2 += v2 * v2; s3 += v3 * v3;
  }
  for (; i < n; i += stride) {
    const double v = w[i];
    s0 += v * v;
  }
  double s = (s0 + s1) + (s2 + s3);
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[l * ppl + p] = (red[0] + red[1]) + (red[2] + red[3]);
}

// one wave per entry: lane i adds partials i, i + 64, ... in order, then a
// fixed butterfly over the lanes (deterministic)
__global__ __launch_bounds__(64) void wnorm_final_kernel(const double* __restrict__ part, int ppl, int nl,
                                                         double* __restrict__ norm2, float* __restrict__ denom,
                                                         int max_norm) {
  // entries [0, nl/2) are weights (clip denominators); the rest only get norm2
  const int l = blockIdx.x, lane = threadIdx.x;
  double s = 0.0;
  for (int p = lane; p < ppl; p += 64) s += part[l * ppl + p];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) {
    norm2[l] = s;
    if (l < nl / 2) denom[l] = max_norm ? fmaxf((float)sqrt(s), 1.0f) : 1.0f;
  }
}

void launch_wnorm(const float* params, const int64_t* offs, const int64_t* sizes, int nl,
                  double* part, int ppl, double* norm2, float* denom, int max_norm, hipStream_t s) {
  hipLaunchKernelGGL(wnorm_part_kernel, dim3(ppl, nl), dim3(256), 0, s, params, offs, sizes, part,
                     ppl);
  hipLaunchKernelGGL(wnorm_final_kernel, dim3(nl), dim3(64), 0, s, part, ppl, nl, norm2, denom,
                     max_norm);
}

// Packed weight blocks for the MFMA kernels are fragment-packed
// (lcn_internal.h frag_ix): block[n][k] with n the output and k the reduction
// index of the GEMM that reads it.

// hidden layer: one workgroup per 64x64 block (si, so) of W_e:
// fwd block [n = q][k = p] (z = a.We), bwd block [n = p][k = q] (da = dz.We^T)
// (all hidden layers in one launch: blockIdx.y picks the layer)
__global__ __launch_bounds__(256) void wprep_hidden_kernel(const float* __restrict__ params,
                                                           const WPrepHidden* __restrict__ items,
                                                           int ld, const int2* __restrict__ blk,
                                                           int spj, const float* __restrict__ M,
                                                           const float* __restrict__ denom) {
  const int b = blockIdx.x;
  const WPrepHidden it = items[blockIdx.y];
  const float* __restrict__ W = params + it.w_off;
  float* __restrict__ fwd = it.fwd;
  float* __restrict__ bwd = it.bwd;
  const int2 sb = blk[b];
  const float m = M[(sb.x / spj) * kJ + (sb.y / spj)];
  const float dn = denom[it.layer];
  for (int e = threadIdx.x; e < 4096; e += 256) {
    const int p = e >> 6, q = e & 63;
    const float v = (W[(size_t)(sb.x * 64 + p) * ld + sb.y * 64 + q] / dn) * m;
    bwd[(size_t)b * 4096 + frag_ix(p, q)] = v;
    fwd[(size_t)b * 4096 + frag_ix(q, p)] = v;
  }
}

// lift (K = 17*C padded to 64): block so [n = f][k] = W_e[k][so*64 + f], zero for k >= 17*C
__global__ __launch_bounds__(256) void wprep_lift_kernel(const float* __restrict__ W, int C,
                                                         int nslab, int spj,
                                                         const float* __restrict__ M,
                                                         const float* __restrict__ denom, int layer,
                                                         float* __restrict__ blk) {
  const int so = blockIdx.x, ld = nslab * 64;
  const float dn = denom[layer];
  for (int e = threadIdx.x; e < 4096; e += 256) {
    const int k = e >> 6, f = e & 63;  // coalesced W reads along f
    float v = 0.f;
    if (k < kJ * C) v = (W[(size_t)k * ld + so * 64 + f] / dn) * M[(k / C) * kJ + so / spj];
    blk[(size_t)so * 4096 + frag_ix(f, k)] = v;
  }
}

// output (N = 51 padded to 64): block si fwd [n = c'][k = p], bwd [n = p][k = c'],
// = W_e[si*64 + p][c'], zero for c' >= 51
__global__ __launch_bounds__(256) void wprep_out_kernel(const float* __restrict__ W, int F,
                                                        const float* __restrict__ M,
                                                        const float* __restrict__ denom, int layer,
                                                        float* __restrict__ fwd,
                                                        float* __restrict__ bwd) {
  constexpr int N = kJ * 3;
  const int si = blockIdx.x;
  const float dn = denom[layer];
  for (int e = threadIdx.x; e < 4096; e += 256) {
    const int p = e >> 6, c = e & 63;  // coalesced W reads along c
    const int r = si * 64 + p;
    float v = 0.f;
    if (c < N) v = (W[(size_t)r * N + c] / dn) * M[(r / F) * kJ + c / 3];
    bwd[(size_t)si * 4096 + frag_ix(p, c)] = v;
    fwd[(size_t)si * 4096 + frag_ix(c, p)] = v;
  }
}

void launch_wprep_hidden(const float* params, const WPrepHidden* items, int n_layers, int ld,
                         const int2* blk, int nblk, int spj, const float* M, const float* denom,
                         hipStream_t s) {
  if (n_layers <= 0) return;
  hipLaunchKernelGGL(wprep_hidden_kernel, dim3(nblk, n_layers), dim3(256), 0, s, params, items, ld, blk,
                     spj, M, denom);
}

void launch_wprep(const float* params, const WLayer& L, const float* M, const float* denom,
                  int layer, hipStream_t s) {
  const float* W = params + L.w_off;
  if (L.kind == 0) {
    const int nslab = L.nout / 64, spj = L.fout / 64;
    hipLaunchKernelGGL(wprep_lift_kernel, dim3(nslab), dim3(256), 0, s, W, L.fin, nslab, spj, M,
                       denom, layer, L.blk_fwd);
  } else {
    const int nslab = L.kin / 64;
    hipLaunchKernelGGL(wprep_out_kernel, dim3(nslab), dim3(256), 0, s, W, L.fin, M, denom, layer,
                       L.blk_fwd, L.blk_bwd);
  }
}

// blocksum[l][i][j] = sum over joint block (i, j) of dWe * W   (float64)
__global__ __launch_bounds__(256) void wdot_kernel(const float* __restrict__ rg,
                                                   const float* __restrict__ params,
                                                   const int64_t* __restrict__ offs,
                                                   const int* __restrict__ kin,
                                                   const int* __restrict__ nout,
                                                   double* __restrict__ blocksum) {
  __shared__ double red[4];
  const int l = blockIdx.y, ij = blockIdx.x, i = ij / kJ, j = ij - i * kJ;
  const int K = kin[l], N = nout[l], fin = K / kJ, fout = N / kJ;
  const float* g = rg + offs[l];
  const float* w = params + offs[l];
  double s = 0.0;
  const int n = fin * fout;
  for (int e = threadIdx.x; e < n; e += 256) {
    const int p = e / fout, q = e - p * fout;
    const size_t o = (size_t)(i * fin + p) * N + j * fout + q;
    s += (double)g[o] * (double)w[o];
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) blocksum[l * kJ * kJ + ij] = (red[0] + red[1]) + (red[2] + red[3]);
}

void launch_wdot(const float* rg, const float* params, const int64_t* offs, const int* kin,
                 const int* nout, int nl, double* blocksum, hipStream_t s) {
  hipLaunchKernelGGL(wdot_kernel, dim3(kJ * kJ, nl), dim3(256), 0, s, rg, params, offs, kin, nout,
                     blocksum);
}

// dM[i,j] = sum_l blocksum_l[i,j] / denom_l  (= sum dWe * W_c);
// <dW_c, W>_l = sum_ij M[i,j] blocksum_l[i,j];  lcoef[l] = (1/n_l, <dW_c,W>_l / n_l^3)
// when clipping is active, else (1, 0);  dV = S (.) (dS - sum_i S dS), dS = dM (.) C.
__global__ __launch_bounds__(320) void maskgrad_kernel(const double* __restrict__ bs, int nl,
                                                       const float* __restrict__ M,
                                                       const float* __restrict__ S,
                                                       const float* __restrict__ C, int learnable,
                                                       const float* __restrict__ denom,
                                                       const double* __restrict__ norm2, int max_norm,
                                                       float* __restrict__ dV,
                                                       float* __restrict__ lcoef) {
  __shared__ double dS[kJ * kJ];
  const int t = threadIdx.x;
  // one wave per layer: lane i adds entries i, i + 64, ..., then a fixed
  // butterfly over the lanes (deterministic)
  for (int l = t >> 6; l < nl; l += 320 / 64) {
    const int lane = t & 63;
    double dot = 0.0;
    for (int e = lane; e < kJ * kJ; e += 64) dot += (double)M[e] * bs[l * kJ * kJ + e];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dot += __shfl_xor(dot, off);
    if (lane == 0) {
      const double n = sqrt(norm2[l]);
      if (max_norm && n > 1.0) {
        lcoef[2 * l] = (float)(1.0 / n);
        lcoef[2 * l + 1] = (float)(dot / (n * n * n));
      } else {
        lcoef[2 * l] = 1.f;
        lcoef[2 * l + 1] = 0.f;
      }
    }
  }
  if (!learnable) return;
  if (t < kJ * kJ) {
    double dm = 0.0;
    for (int l = 0; l < nl; ++l) dm += bs[l * kJ * kJ + t] / (double)denom[l];
    dS[t] = C[t] != 0.f ? dm : 0.0;
  }
  __syncthreads();
  if (t < kJ * kJ) {
    const int j = t % kJ;
    double col = 0.0;
    for (int i = 0; i < kJ; ++i) col += (double)S[i * kJ + j] * dS[i * kJ + j];
    dV[t] = (float)((double)S[t] * (dS[t] - col));
  }
}

void launch_maskgrad(const double* blocksum, int nl, const float* M, const float* S,
                     const float* Cmat, int learnable, const float* denom, const double* norm2,
                     int max_norm, float* dV, float* lcoef, hipStream_t s) {
  hipLaunchKernelGGL(maskgrad_kernel, dim3(1), dim3(320), 0, s, blocksum, nl, M, S, Cmat, learnable,
                     denom, norm2, max_norm, dV, lcoef);
}

// Fused gradient finish + Adam over the flat parameter vector.  Weights get
// the clip/mask backward  g = dWe * M[i,j] / n - c_l * W .
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ theta, float* __restrict__ m,
                                                   float* __restrict__ v,
                                                   const float* __restrict__ rg,
                                                   float* __restrict__ gout,
                                                   const AdamSeg* __restrict__ segs,
                                                   const int64_t* __restrict__ seg_start, int nseg,
                                                   const float* __restrict__ M,
                                                   const float* __restrict__ lcoef, float reg,
                                                   const float* __restrict__ lr_t_dev, float beta1,
                                                   float beta2, float eps, int update) {
  const int64_t b = blockIdx.x;
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (seg_start[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const AdamSeg sg = segs[lo];
  const int64_t base = (b - seg_start[lo]) * 1024;
  const float omb1 = 1.f - beta1, omb2 = 1.f - beta2;
  // lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t), computed by the host per
  // step and written to device memory (so a captured step graph replays it)
  const float lr_t = *lr_t_dev;
  for (int k = 0; k < 4; ++k) {
    const int64_t e = base + k * 256 + threadIdx.x;
    if (e >= sg.size) break;
    const int64_t o = sg.off + e;
    const float th = theta[o];
    float g = rg[o];
    if (sg.kind == 1) {
      const int r = (int)(e / sg.cols), c = (int)(e - (int64_t)r * sg.cols);
      const float mv = M[(r / sg.fin) * kJ + c / sg.fout];
      g = (g * mv) * lcoef[2 * sg.layer] - lcoef[2 * sg.layer + 1] * th;
    }
    if (sg.reg) g += reg * th;
    if (gout) gout[o] = g;
    if (update) {
      float mm = m[o], vv = v[o];
      mm += (g - mm) * omb1;
      vv += (g * g - vv) * omb2;
      m[o] = mm;
      v[o] = vv;
      theta[o] = th - (mm * lr_t) / (sqrtf(vv) + eps);
    }
  }
}

void launch_adam(float* theta, float* m, float* v, const float* rg, float* gout,
                 const AdamSeg* segs, const int64_t* seg_block_start, int nseg,
                 int64_t total_blocks, const float* M, const float* lcoef, float reg,
                 const float* lr_t_dev, float beta1, float beta2, float eps, int update, hipStream_t s) {
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)total_blocks), dim3(256), 0, s, theta, m, v, rg,
                     gout, segs, seg_block_start, nseg, M, lcoef, reg, lr_t_dev, beta1, beta2, eps,
                     update);
}

}  // namespace lcn
