// Device helpers shared by the block-sparse GEMM kernels (gfx950).
#pragma once
#include "lcn_internal.h"

namespace lcn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  // blocks b, b+8, ... share an XCD; give each XCD a contiguous range of work ids
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// tf.nn.leaky_relu: max(alpha * u, u)  (alpha < 1)
__device__ __forceinline__ float leaky(float u, float alpha) { return fmaxf(u * alpha, u); }

// BN apply + LeakyReLU: leaky(z * scale + shift)  (tf.nn.batch_normalization, tf.nn.leaky_relu)
__device__ __forceinline__ float4 bnact4(float4 v, float4 sc, float4 sh, float alpha) {
  v.x = leaky(fmaf(v.x, sc.x, sh.x), alpha);
  v.y = leaky(fmaf(v.y, sc.y, sh.y), alpha);
  v.z = leaky(fmaf(v.z, sc.z, sh.z), alpha);
  v.w = leaky(fmaf(v.w, sc.w, sh.w), alpha);
  return v;
}

// The same with the tables pre-scaled by a = (1 + alpha) / 2 and ba = (1 - alpha) / (1 + alpha):
// leaky(u) = a u + ((1 - alpha) / 2) |u| = u' + ba |u'| for u' = a u -- two operations an element
__device__ __forceinline__ float4 bnact4_scaled(float4 v, float4 sc, float4 sh, float ba) {
  v.x = fmaf(v.x, sc.x, sh.x); v.x = fmaf(fabsf(v.x), ba, v.x);
  v.y = fmaf(v.y, sc.y, sh.y); v.y = fmaf(fabsf(v.y), ba, v.y);
  v.z = fmaf(v.z, sc.z, sh.z); v.z = fmaf(fabsf(v.z), ba, v.z);
  v.w = fmaf(v.w, sc.w, sh.w); v.w = fmaf(fabsf(v.w), ba, v.w);
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

// the same with the slope folded into the coefficient: dz = (u > 0 ? c1 : c1 alpha) dh + (c3 z + c2)
__device__ __forceinline__ float bnback1_sel(float dh, float z, float sc, float sh, float c1, float c1a, float c2,
                                             float c3) {
  const float u = fmaf(z, sc, sh);
  return fmaf(u > 0.f ? c1 : c1a, dh, fmaf(c3, z, c2));
}
__device__ __forceinline__ float4 bnback4_sel(float4 dh, float4 z, const BnBackCoef& c, float4 c1a) {
  float4 r;
  r.x = bnback1_sel(dh.x, z.x, c.sc.x, c.sh.x, c.c1.x, c1a.x, c.c2.x, c.c3.x);
  r.y = bnback1_sel(dh.y, z.y, c.sc.y, c.sh.y, c.c1.y, c1a.y, c.c2.y, c.c3.y);
  r.z = bnback1_sel(dh.z, z.z, c.sc.z, c.sh.z, c.c1.z, c1a.z, c.c2.z, c.c3.z);
  r.w = bnback1_sel(dh.w, z.w, c.sc.w, c.sh.w, c.c1.w, c1a.w, c.c2.w, c.c3.w);
  return r;
}

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

// Reduce-scatter over the 32 lanes of each half-wave: v[i] (i < 32) per lane
// in, and on return v[0] of lane l holds sum over the 32 lanes of l's half of
// v[l & 31].  31 butterfly exchanges (xor 16, 8, 4, 2, 1) instead of 32 full
// reductions; fixed order, deterministic.
template <int N>
__device__ __forceinline__ void rs_step(float (&v)[32], int lane) {
  constexpr int H = N / 2;
  const bool up = (lane & H) != 0;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const float keep = up ? v[i + H] : v[i];
    const float send = up ? v[i] : v[i + H];
    v[i] = keep + __shfl_xor(send, H);
  }
}
__device__ __forceinline__ float halfwave_reduce_scatter(float (&v)[32], int lane) {
  rs_step<32>(v, lane);
  rs_step<16>(v, lane);
  rs_step<8>(v, lane);
  rs_step<4>(v, lane);
  rs_step<2>(v, lane);
  return v[0];
}

// feature (0..63 within the output slab) of accumulator value index i (0..31:
// acc0[0..15] then acc1[0..15]) in lane half h
__device__ __forceinline__ int acc_feature(int i, int h) {
  return 32 * (i >> 4) + 8 * ((i >> 2) & 3) + 4 * h + (i & 3);
}

}  // namespace lcn
