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

// Epilogue of a 128-row x 64-column tile computed by 4 waves of 32 x 64
// (acc0: columns 0-31, acc1: 32-63).  C/D map of the 32x32 MFMA: column =
// lane&31, row = (k&3) + 8(k>>2) + 4(lane>>5).  Adds bias (forward) or the
// residual gradient (backward), stores, and writes the BN partials of the
// tile: (sum, sum of squared deviations about the tile mean) per column.
__device__ __forceinline__ void gemm_epilogue_32x64(const GemmArgs& a, f32x16& acc0, f32x16& acc1,
                                                    int rt, int so, int row0, int w, int lr, int h,
                                                    float* smem) {
  const int B = a.B, ldy = a.ldy;
  float* __restrict__ Y = a.Y;
  const float* __restrict__ addsrc = a.addsrc;
  float2* __restrict__ stat = a.stat;
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
  if (stat == nullptr) return;
  const int nval = min(128, B - row0);
  s0 += __shfl_xor(s0, 32);
  s1 += __shfl_xor(s1, 32);
  __syncthreads();
  float* red = smem;  // [4][64] sums, then [4][64] m2
  if (h == 0) { red[w * 64 + lr] = s0; red[w * 64 + 32 + lr] = s1; }
  __syncthreads();
  const float tot0 = (red[lr] + red[64 + lr]) + (red[128 + lr] + red[192 + lr]);
  const float tot1 = (red[32 + lr] + red[96 + lr]) + (red[160 + lr] + red[224 + lr]);
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
  m0 += __shfl_xor(m0, 32);
  m1 += __shfl_xor(m1, 32);
  float* red2 = smem + 256;
  if (h == 0) { red2[w * 64 + lr] = m0; red2[w * 64 + 32 + lr] = m1; }
  __syncthreads();
  if (w == 0 && h == 0) {
    const float q0 = (red2[lr] + red2[64 + lr]) + (red2[128 + lr] + red2[192 + lr]);
    const float q1 = (red2[32 + lr] + red2[96 + lr]) + (red2[160 + lr] + red2[224 + lr]);
    stat[(size_t)rt * ldy + ncol0] = make_float2(tot0, q0);
    stat[(size_t)rt * ldy + ncol1] = make_float2(tot1, q1);
  }
}

// Epilogue of a 256-row x 64-column tile: 4 waves x 64 rows; per wave acc0x
// covers its rows 0-31 and acc1x rows 32-63 (x = column half).
__device__ __forceinline__ void gemm_epilogue_64x64(const GemmArgs& a, f32x16& acc00, f32x16& acc01,
                                                    f32x16& acc10, f32x16& acc11, int rt, int so,
                                                    int row0, int w, int lr, int h, float* smem) {
  const int B = a.B, ldy = a.ldy;
  float* __restrict__ Y = a.Y;
  const float* __restrict__ addsrc = a.addsrc;
  float2* __restrict__ stat = a.stat;
  const int ncol0 = so * kSlab + lr, ncol1 = ncol0 + 32;
  const float bias0 = a.bias ? a.bias[ncol0] : 0.f;
  const float bias1 = a.bias ? a.bias[ncol1] : 0.f;
  const int rb = row0 + 64 * w + 4 * h;
  float s0 = 0.f, s1 = 0.f;
#define EPI_STORE(ACC0, ACC1, ROFF)                                         \
  _Pragma("unroll") for (int k = 0; k < 16; ++k) {                         \
    const int row = rb + (ROFF) + (k & 3) + 8 * (k >> 2);                  \
    float v0 = ACC0[k] + bias0, v1 = ACC1[k] + bias1;                      \
    if (row < B) {                                                         \
      const size_t o = (size_t)row * ldy;                                  \
      if (addsrc) { v0 += addsrc[o + ncol0]; v1 += addsrc[o + ncol1]; }    \
      Y[o + ncol0] = v0;                                                   \
      Y[o + ncol1] = v1;                                                   \
      s0 += v0;                                                            \
      s1 += v1;                                                            \
    }                                                                      \
    ACC0[k] = v0;                                                          \
    ACC1[k] = v1;                                                          \
  }
  EPI_STORE(acc00, acc01, 0)
  EPI_STORE(acc10, acc11, 32)
#undef EPI_STORE
  if (stat == nullptr) return;
  const int nval = min(256, B - row0);
  s0 += __shfl_xor(s0, 32);
  s1 += __shfl_xor(s1, 32);
  __syncthreads();
  float* red = smem;  // [4][64] sums, then [4][64] m2
  if (h == 0) { red[w * 64 + lr] = s0; red[w * 64 + 32 + lr] = s1; }
  __syncthreads();
  const float tot0 = (red[lr] + red[64 + lr]) + (red[128 + lr] + red[192 + lr]);
  const float tot1 = (red[32 + lr] + red[96 + lr]) + (red[160 + lr] + red[224 + lr]);
  const float mean0 = tot0 / (float)nval, mean1 = tot1 / (float)nval;
  float m0 = 0.f, m1 = 0.f;
#define EPI_M2(ACC0, ACC1, ROFF)                                            \
  _Pragma("unroll") for (int k = 0; k < 16; ++k) {                         \
    const int row = rb + (ROFF) + (k & 3) + 8 * (k >> 2);                  \
    if (row < B) {                                                         \
      const float d0 = ACC0[k] - mean0, d1 = ACC1[k] - mean1;              \
      m0 = fmaf(d0, d0, m0);                                               \
      m1 = fmaf(d1, d1, m1);                                               \
    }                                                                      \
  }
  EPI_M2(acc00, acc01, 0)
  EPI_M2(acc10, acc11, 32)
#undef EPI_M2
  m0 += __shfl_xor(m0, 32);
  m1 += __shfl_xor(m1, 32);
  float* red2 = smem + 256;
  if (h == 0) { red2[w * 64 + lr] = m0; red2[w * 64 + 32 + lr] = m1; }
  __syncthreads();
  if (w == 0 && h == 0) {
    const float q0 = (red2[lr] + red2[64 + lr]) + (red2[128 + lr] + red2[192 + lr]);
    const float q1 = (red2[32 + lr] + red2[96 + lr]) + (red2[160 + lr] + red2[224 + lr]);
    stat[(size_t)rt * ldy + ncol0] = make_float2(tot0, q0);
    stat[(size_t)rt * ldy + ncol1] = make_float2(tot1, q1);
  }
}

}  // namespace lcn
