// Epilogue of the block-sparse forward / backward-data GEMM kernels
// (gemm_bs.hip: one output slab per workgroup; gemm_pair.hip: two): residual
// add, output store and the per-128-row BN partials of one 64-wide output slab.
#pragma once
#include "gemm_common.h"

namespace lcn {

typedef float v4f_t __attribute__((ext_vector_type(4)));
typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
// one 16-byte buffer load: scalar resource, one 32-bit lane offset, scalar offset
#define BUFLD(RES, VOFF, SOFF)                                                         \
  ({                                                                                   \
    const v4f_t v_ = __builtin_bit_cast(v4f_t, __builtin_amdgcn_raw_buffer_load_b128((RES), (VOFF), (SOFF), 0)); \
    make_float4(v_.x, v_.y, v_.z, v_.w);                                               \
  })

// EPI_BNBACK with the dropout of the layer below: a separate instance, since
// the mask hash costs the plain kernel registers (it spilled)
constexpr int kEpiBnBackDrop = 3;

// float4 offset of the BN tables / epilogue constants / wave merge in LDS: after
// the weight double buffer (2 x 16 KB) and the epilogue's 8 KB per wave
constexpr int kTabOff = kGemmWaves > 4 ? kGemmWaves * 512 : 2048;

// EPI_BNBACK: per-channel constants of output slab `so` -> LDS table [4][64]
// (scale, shift, mean, rstd of the BN layer below); the first four waves fill it
__device__ __forceinline__ void epi_fill_table(const GemmArgs& a, float* ptab, int so) {
  const int pk = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ch = (so % (a.epi_F / kSlab)) * kSlab + lane;
  const float* src = pk == 0 ? a.epi_scale : pk == 1 ? a.epi_shift : pk == 2 ? a.epi_mean : a.epi_rstd;
  if (pk < 4) ptab[threadIdx.x] = src[ch];
}

// Every wave of the workgroup calls this with its 32-row x 64-column
// accumulator tile (acc0: features 0..31, acc1: 32..63 of output slab `so` of
// row tile `rt`; `live` false: a wave past the last row tile, which only takes
// part in the barriers).  Y = acc (+ addsrc); then, per 128-row group `rtg`,
// either the BN forward partials of the output (sum, M2 about the group mean)
// or the BN backward partials of the layer below (sum du, sum du * zhat):
// column sums per wave through LDS, merged across the waves.
//   Wl    the workgroup's LDS: the (then free) weight buffers serve as the
//         per-wave transpose space, 8 KB a wave
//   ptab  EPI_BNBACK: the table epi_fill_table wrote for `so`
//   comb  [waves][64][3] floats of LDS for the wave merge
// Contains workgroup barriers: the call must be workgroup-uniform.
template <int EPI>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& a, float4* Wl, const float* ptab, float* comb, int rtg,
                                              int rt, bool live, int so, const f32x16& acc0, const f32x16& acc1) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int xlo = lane * 16;
  const int S_out = a.S_out, ncols = S_out * kSlab;
  const float al = a.alpha;
#define OUT_RES(PTR) \
  __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)(PTR) + (size_t)rt * S_out * 8192), 0, S_out * 8192, 0x00020000)
  float4 zp0, zp1, zp2, zp3, zp4, zp5, zp6, zp7;
  if constexpr (EPI == EPI_BNBACK || EPI == kEpiBnBackDrop) {
    // z of the layer below, issued before the output stores so its latency
    // overlaps them (keeping it live through the loop would cost 32 VGPRs,
    // i.e. a wave per SIMD of occupancy)
#ifdef EXP_DX_NOZ  // diagnostic: the epilogue's z tile comes from one hot tile (no HBM traffic, no miss latency)
    const __amdgpu_buffer_rsrc_t zres = __builtin_amdgcn_make_buffer_rsrc((void*)a.epi_z, 0, S_out * 8192, 0x00020000);
    const int zo = 0;
#else
    const __amdgpu_buffer_rsrc_t zres = OUT_RES(a.epi_z);
    const int zo = so * 8192;
#endif
    zp0 = BUFLD(zres, xlo, zo);        zp1 = BUFLD(zres, xlo + 1024, zo);
    zp2 = BUFLD(zres, xlo + 2048, zo); zp3 = BUFLD(zres, xlo + 3072, zo);
    zp4 = BUFLD(zres, xlo, zo + 4096);        zp5 = BUFLD(zres, xlo + 1024, zo + 4096);
    zp6 = BUFLD(zres, xlo + 2048, zo + 4096); zp7 = BUFLD(zres, xlo + 3072, zo + 4096);
  }
  float v[32];
#pragma unroll
  for (int k = 0; k < 16; ++k) { v[k] = acc0[k]; v[16 + k] = acc1[k]; }
  // the residual is added after the loop, its loads in flight together with
  // the epilogue's z (what the residual costs the dX GEMM is its 285 MB of
  // traffic: 781 us with it, 757 us without; loading it ahead of the loop or
  // after it measured the same, 784 vs 781 us)
  if (a.addsrc) {  // Y = acc + addsrc (addsrc may be Y itself: each lane reads what it then writes)
    const __amdgpu_buffer_rsrc_t rres = OUT_RES(a.addsrc);
    float4 rq[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) rq[q] = BUFLD(rres, xlo + (q & 3) * 1024, so * 8192 + (q >> 2) * 4096);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      v[4 * q + 0] += rq[q].x; v[4 * q + 1] += rq[q].y; v[4 * q + 2] += rq[q].z; v[4 * q + 3] += rq[q].w;
    }
  }
  if (live) {
    const __amdgpu_buffer_rsrc_t yres = OUT_RES(a.Y);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const v4f_t o_ = {v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};  // chunk q: features 8q + 4h .. +3
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, o_), yres, xlo + (q & 3) * 1024,
                                             so * 8192 + (q >> 2) * 4096, 0);
    }
  }
#undef OUT_RES
  if constexpr (EPI == EPI_NONE) return;
  // Column partials of the wave's 32x64 tile through its 8 KB of the (now
  // free) weight LDS: the wave writes float4 chunks with a lane swizzle
  // (position l ^ (2q + (l>>5)) of chunk q) that makes the column-wise reads
  // bank-conflict free; lane c then sums column c over the tile's rows.
  __syncthreads();  // all waves are done with the weight buffers (and with comb)
  // Each wave transposes through its own 8 KB: a wave's LDS operations execute
  // in issue order, so its column reads see its own writes (and a later write
  // pass follows the earlier reads) without a workgroup barrier; the compiler
  // only has to keep the program order.
#define EPI_SYNC() __builtin_amdgcn_wave_barrier()
  float* red = (float*)Wl + w * 2048;
  const int c = lane, cg = c >> 3, chh = (c >> 2) & 1, cs = c & 3;
  const int n = live ? min(kRT, a.B - rt * kRT) : 0;  // valid rows of the tile
  float2* stat = a.stat + (size_t)rtg * ncols + so * kSlab + c;
  auto put = [&](int q, float x0, float x1, float x2, float x3) {
    const int pos = lane ^ (2 * q + h);
    *(float4*)(red + (q * 64 + pos) * 4) = make_float4(x0, x1, x2, x3);
  };
  // value of row r of column c (r < 32)
  auto get = [&](int r) {
    const int l = r + 32 * chh;
    return red[(cg * 64 + (l ^ (2 * cg + chh))) * 4 + cs];
  };
  if constexpr (EPI == EPI_BNFWD) {
#pragma unroll
    for (int q = 0; q < 8; ++q) put(q, v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    EPI_SYNC();
    float sum = 0.f, mean = 0.f, m2 = 0.f;
    if (n == kRT) {  // full tile: 16 reads in flight at a time; / 32 is exact as * (1/32)
#pragma unroll
      for (int r0 = 0; r0 < kRT; r0 += 16) {
        float col[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) col[r] = get(r0 + r);
#pragma unroll
        for (int r = 0; r < 16; ++r) sum += col[r];
      }
      mean = sum * (1.f / kRT);
#pragma unroll
      for (int r0 = 0; r0 < kRT; r0 += 16) {
        float col[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) col[r] = get(r0 + r);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = col[r] - mean;
          m2 = fmaf(d, d, m2);
        }
      }
    } else {
      for (int r = 0; r < n; ++r) sum += get(r);
      mean = n > 0 ? sum / (float)n : 0.f;
      for (int r = 0; r < n; ++r) {
        const float d = get(r) - mean;
        m2 = fmaf(d, d, m2);
      }
    }
    comb[(w * 64 + c) * 3 + 0] = sum;
    comb[(w * 64 + c) * 3 + 1] = m2;
    comb[(w * 64 + c) * 3 + 2] = (float)n;
    __syncthreads();
    if (w == 0) {  // Chan et al. merge of the row tiles: (sum, M2 about the group mean)
      float S = 0.f, N = 0.f;
#pragma unroll
      for (int i = 0; i < kGemmWaves; ++i) {
        S += comb[(i * 64 + c) * 3 + 0];
        N += comb[(i * 64 + c) * 3 + 2];
      }
      const float mu = S / N;
      float M2 = 0.f;
#pragma unroll
      for (int i = 0; i < kGemmWaves; ++i) {
        const float ni = comb[(i * 64 + c) * 3 + 2];
        if (ni > 0.f) {
          const float d = comb[(i * 64 + c) * 3 + 0] / ni - mu;
          M2 += comb[(i * 64 + c) * 3 + 1] + ni * d * d;
        }
      }
      *stat = make_float2(S, M2);
    }
    return;
  } else {
    // EPI_BNBACK: du = dh * leaky'(u(z)), zhat = (z - mean) * rstd of the layer
    // below; pass 0 reduces du, pass 1 du * zhat
    // dropout of the layer below (tf.nn.dropout's gradient: dh * mask * scale),
    // applied to the partials only -- the stored dh stays the incoming gradient
    if constexpr (EPI == kEpiBnBackDrop) {
      const int64_t row = (int64_t)rt * kRT + (lane & 31);
      const Dropout dr = drop_resolve(a.epi_drop);
#pragma unroll
      for (int i = 0; i < 32; ++i) v[i] = drop_apply(dr, row, so * kSlab + acc_feature(i, h), v[i]);
    }
    // column c summed over the tile's n rows in row order (a full tile with
    // 16 LDS reads in flight at a time)
    auto colsum = [&](int nr) {
      float acc = 0.f;
      if (nr == kRT) {
#pragma unroll
        for (int r0 = 0; r0 < kRT; r0 += 16) {
          float col[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) col[r] = get(r0 + r);
#pragma unroll
          for (int r = 0; r < 16; ++r) acc += col[r];
        }
      } else {
        for (int r = 0; r < nr; ++r) acc += get(r);
      }
      return acc;
    };
    float P_ = 0.f, Q_ = 0.f;
#ifdef EXP_DX_NOSUM  // diagnostic: no column-sum passes (the z tile is still loaded and consumed)
    P_ = zp0.x + zp1.x + zp2.x + zp3.x + zp4.x + zp5.x + zp6.x + zp7.x + v[lane & 31];
#else
    {
      const float4 zq[8] = {zp0, zp1, zp2, zp3, zp4, zp5, zp6, zp7};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 z4 = zq[q];
        const int ch = 8 * q + 4 * h;
        const float4 sc = *(const float4*)(ptab + ch), sh = *(const float4*)(ptab + 64 + ch);
        v[4 * q + 0] = fmaf(z4.x, sc.x, sh.x) > 0.f ? v[4 * q + 0] : v[4 * q + 0] * al;
        v[4 * q + 1] = fmaf(z4.y, sc.y, sh.y) > 0.f ? v[4 * q + 1] : v[4 * q + 1] * al;
        v[4 * q + 2] = fmaf(z4.z, sc.z, sh.z) > 0.f ? v[4 * q + 2] : v[4 * q + 2] * al;
        v[4 * q + 3] = fmaf(z4.w, sc.w, sh.w) > 0.f ? v[4 * q + 3] : v[4 * q + 3] * al;
        put(q, v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
      }
      EPI_SYNC();
      P_ = colsum(n);
      EPI_SYNC();
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 z4 = zq[q];
        const int ch = 8 * q + 4 * h;
        const float4 mu = *(const float4*)(ptab + 128 + ch), rs = *(const float4*)(ptab + 192 + ch);
        put(q, v[4 * q] * ((z4.x - mu.x) * rs.x), v[4 * q + 1] * ((z4.y - mu.y) * rs.y),
            v[4 * q + 2] * ((z4.z - mu.z) * rs.z), v[4 * q + 3] * ((z4.w - mu.w) * rs.w));
      }
      EPI_SYNC();
      Q_ = colsum(n);
    }
#endif
    comb[(w * 64 + c) * 3 + 0] = P_;
    comb[(w * 64 + c) * 3 + 1] = Q_;
    __syncthreads();
    if (w == 0) {
      float P = 0.f, Q = 0.f;
#pragma unroll
      for (int i = 0; i < kGemmWaves; ++i) {
        P += comb[(i * 64 + c) * 3 + 0];
        Q += comb[(i * 64 + c) * 3 + 1];
      }
      *stat = make_float2(P, Q);
    }
  }
#undef EPI_SYNC
}

}  // namespace lcn
