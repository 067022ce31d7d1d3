// Device helpers shared by the block-sparse GEMM kernels (gfx950).
#pragma once
#include "lcn_internal.h"

namespace lcn {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int LDA = 68;  // LDS row stride in floats: +4 makes the ds_read_b128 fragment reads conflict-free

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  // blocks b, b+8, ... share an XCD; give each XCD a contiguous range of work ids
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

__device__ __forceinline__ float leaky(float u, float alpha) { return u > 0.f ? u : u * alpha; }

// BN apply + LeakyReLU: leaky(z * scale + shift)  (tf.nn.batch_normalization, tf.nn.leaky_relu)
__device__ __forceinline__ float4 bnact4(float4 v, float4 sc, float4 sh, float alpha) {
  v.x = leaky(fmaf(v.x, sc.x, sh.x), alpha);
  v.y = leaky(fmaf(v.y, sc.y, sh.y), alpha);
  v.z = leaky(fmaf(v.z, sc.z, sh.z), alpha);
  v.w = leaky(fmaf(v.w, sc.w, sh.w), alpha);
  return v;
}

// BN + LeakyReLU backward:
//   u = scale*z + shift,  du = u > 0 ? dh : alpha*dh,  dz = c1*du + c2 + c3*z
struct BnBackCoef { float4 sc, sh, c1, c2, c3; };

__device__ __forceinline__ BnBackCoef load_bnback_coef(const float* scale, const float* shift,
                                                       const float* c123, int F, int ch) {
  BnBackCoef c;
  c.sc = *(const float4*)(scale + ch);
  c.sh = *(const float4*)(shift + ch);
  c.c1 = *(const float4*)(c123 + ch);
  c.c2 = *(const float4*)(c123 + F + ch);
  c.c3 = *(const float4*)(c123 + 2 * F + ch);
  return c;
}

__device__ __forceinline__ float bnback1(float dh, float z, float sc, float sh, float c1, float c2,
                                         float c3, float alpha) {
  const float u = fmaf(z, sc, sh);
  const float du = u > 0.f ? dh : dh * alpha;
  return fmaf(c1, du, fmaf(c3, z, c2));
}

__device__ __forceinline__ float4 bnback4(float4 dh, float4 z, const BnBackCoef& c, float alpha) {
  float4 r;
  r.x = bnback1(dh.x, z.x, c.sc.x, c.sh.x, c.c1.x, c.c2.x, c.c3.x, alpha);
  r.y = bnback1(dh.y, z.y, c.sc.y, c.sh.y, c.c1.y, c.c2.y, c.c3.y, alpha);
  r.z = bnback1(dh.z, z.z, c.sc.z, c.sh.z, c.c1.z, c.c2.z, c.c3.z, alpha);
  r.w = bnback1(dh.w, z.w, c.sc.w, c.sh.w, c.c1.w, c.c2.w, c.c3.w, alpha);
  return r;
}

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

// 4 k-steps (one float4 of A and of two B columns) into two 32x32 accumulators
#define MFMA_STEP4(AV, B0, B1, ACC0, ACC1)   \
  ACC0 = MFMA32((AV).x, (B0).x, ACC0);       \
  ACC1 = MFMA32((AV).x, (B1).x, ACC1);       \
  ACC0 = MFMA32((AV).y, (B0).y, ACC0);       \
  ACC1 = MFMA32((AV).y, (B1).y, ACC1);       \
  ACC0 = MFMA32((AV).z, (B0).z, ACC0);       \
  ACC1 = MFMA32((AV).z, (B1).z, ACC1);       \
  ACC0 = MFMA32((AV).w, (B0).w, ACC0);       \
  ACC1 = MFMA32((AV).w, (B1).w, ACC1);

// Sum a per-lane value over the 128 rows of the tile for the lane's column:
// the two half-waves, then the 4 waves through LDS (fixed order).
__device__ __forceinline__ float tile_colsum(float v, float* red, int w, int lr, int h, int half) {
  v += __shfl_xor(v, 32);
  if (h == 0) red[w * 64 + half * 32 + lr] = v;
  __syncthreads();
  const int c = half * 32 + lr;
  return (red[c] + red[64 + c]) + (red[128 + c] + red[192 + c]);
}

// Epilogue of a 128-row x 64-column tile computed by 4 waves of 32 x 64
// (acc0: columns 0-31, acc1: 32-63).  C/D map of the 32x32 MFMA: column =
// lane&31, row = (k&3) + 8(k>>2) + 4(lane>>5).  Adds bias (forward) or the
// residual gradient (backward), stores, then writes the tile partials:
//   EPI_BNFWD:  (sum, sum of squared deviations about the tile mean) of Y
//   EPI_BNBACK: (sum du, sum du*zhat) for the BN layer below, with the stored
//               value as its incoming gradient dh
__device__ __forceinline__ void gemm_epilogue_32x64(const GemmArgs& a, f32x16& acc0, f32x16& acc1,
                                                    int rt, int so, int row0, int w, int lr, int h,
                                                    float* smem) {
  const int B = a.B, ldy = a.ldy;
  float* __restrict__ Y = a.Y;
  const float* __restrict__ addsrc = a.addsrc;
  const int ncol0 = so * kSlab + lr, ncol1 = ncol0 + 32;
  const float bias0 = a.bias ? a.bias[ncol0] : 0.f;
  const float bias1 = a.bias ? a.bias[ncol1] : 0.f;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int row = row0 + 32 * w + (k & 3) + 8 * (k >> 2) + 4 * h;
    float v0 = acc0[k] + bias0, v1 = acc1[k] + bias1;
    if (row < B) {
      const size_t o = (size_t)row * ldy;
      if (addsrc) { v0 += addsrc[o + ncol0]; v1 += addsrc[o + ncol1]; }
      Y[o + ncol0] = v0;
      Y[o + ncol1] = v1;
      s0 += v0;
      s1 += v1;
    }
    acc0[k] = v0;
    acc1[k] = v1;
  }
  if (a.epi_mode == EPI_NONE) return;
  float2* __restrict__ stat = a.stat;
  float* red = smem;  // [4][64]
  __syncthreads();    // all waves are done with the staging LDS
  if (a.epi_mode == EPI_BNFWD) {
    const int nval = min(128, B - row0);
    const float tot0 = tile_colsum(s0, red, w, lr, h, 0);
    const float tot1 = tile_colsum(s1, red, w, lr, h, 1);
    const float mean0 = tot0 / (float)nval, mean1 = tot1 / (float)nval;
    float m0 = 0.f, m1 = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int row = row0 + 32 * w + (k & 3) + 8 * (k >> 2) + 4 * h;
      if (row < B) {
        const float d0 = acc0[k] - mean0, d1 = acc1[k] - mean1;
        m0 = fmaf(d0, d0, m0);
        m1 = fmaf(d1, d1, m1);
      }
    }
    __syncthreads();
    const float q0 = tile_colsum(m0, red + 256, w, lr, h, 0);
    const float q1 = tile_colsum(m1, red + 256, w, lr, h, 1);
    if (w == 0 && h == 0) {
      stat[(size_t)rt * ldy + ncol0] = make_float2(tot0, q0);
      stat[(size_t)rt * ldy + ncol1] = make_float2(tot1, q1);
    }
    return;
  }
  // EPI_BNBACK: du = dh * leaky'(u(z)), zhat = (z - mean) * rstd of the layer below
  const float* __restrict__ Z = a.epi_z;
  const int ch0 = ncol0 % a.epi_F, ch1 = ncol1 % a.epi_F;
  const float sc0 = a.epi_scale[ch0], sh0 = a.epi_shift[ch0], mu0 = a.epi_mean[ch0], rs0 = a.epi_rstd[ch0];
  const float sc1 = a.epi_scale[ch1], sh1 = a.epi_shift[ch1], mu1 = a.epi_mean[ch1], rs1 = a.epi_rstd[ch1];
  const float al = a.alpha;
  float p0 = 0.f, p1 = 0.f, q0 = 0.f, q1 = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int row = row0 + 32 * w + (k & 3) + 8 * (k >> 2) + 4 * h;
    if (row < B) {
      const size_t o = (size_t)row * ldy;
      const float z0 = Z[o + ncol0], z1 = Z[o + ncol1];
      const float du0 = fmaf(z0, sc0, sh0) > 0.f ? acc0[k] : acc0[k] * al;
      const float du1 = fmaf(z1, sc1, sh1) > 0.f ? acc1[k] : acc1[k] * al;
      p0 += du0;
      p1 += du1;
      q0 = fmaf(du0, (z0 - mu0) * rs0, q0);
      q1 = fmaf(du1, (z1 - mu1) * rs1, q1);
    }
  }
  const float P0 = tile_colsum(p0, red, w, lr, h, 0);
  const float P1 = tile_colsum(p1, red, w, lr, h, 1);
  __syncthreads();
  const float Q0 = tile_colsum(q0, red + 256, w, lr, h, 0);
  const float Q1 = tile_colsum(q1, red + 256, w, lr, h, 1);
  if (w == 0 && h == 0) {
    stat[(size_t)rt * ldy + ncol0] = make_float2(P0, Q0);
    stat[(size_t)rt * ldy + ncol1] = make_float2(P1, Q1);
  }
}

}  // namespace lcn
