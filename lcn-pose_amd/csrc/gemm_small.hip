// Block-sparse fp32 MFMA GEMM of the LCN layers for SMALL batches (gfx950):
// the same contract as gemm_bs.hip (forward z = a.We + b with BN statistics,
// backward-data dA = dZ.We^T with the BN-backward sums of the layer below),
// for launches whose row tiles are too few to fill the chip.
//
// The reference trains at batch 200 (train.py:21) and 512: 7 / 16 row tiles of
// 32 rows.  gemm_bs_kernel gives a workgroup four row tiles and one output
// slab, so such a launch has 34 / 68 workgroups on 256 CUs and each wave walks
// its 5..17 input slabs one after the other -- the launch is one wave's serial
// chain (~30 us).  Here a workgroup owns ONE row tile x one output slab and
// its four waves split the slab list (wave w takes entries w, w + 4, ...):
// 4 x the workgroups, a quarter of the chain.  There is no reuse of a weight
// block between the waves any more, so each wave reads its weight fragments
// straight from global memory (L2-resident: all workgroups of an output slab
// read the same blocks) into registers, double-buffered one slab ahead with
// the activation fragments -- no LDS and no barrier in the loop.  The four
// partial accumulators are added in wave order through LDS (deterministic),
// and wave 0 runs the epilogue: bias / residual, store, and the per-row-tile
// BN partials (stat[rt][column]; colreduce merges 32-row tiles here, 128-row
// groups after gemm_bs_kernel).
#include "gemm_common.h"

namespace lcn {

namespace {

// one input slab in registers: 8 activation fragments + 16 weight fragments
struct SlabRegs {
  float4 x[8];
  float4 w[16];
};

}  // namespace

template <int PRO, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_bs_small_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) float red[3 * 2048];  // partial accumulators of waves 1..3
  __shared__ __attribute__((aligned(16))) float tab[4 * 64];    // epilogue constants (EPI_BNBACK)
  extern __shared__ __attribute__((aligned(16))) float dyn[];   // BN scale / shift of the operand (PRO_BNACT)
  const int nso = a.n_out_slabs;
  const int rt = blockIdx.x / nso, so = blockIdx.x - rt * nso;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int beg = a.ptr[so], end = a.ptr[so + 1];
  const int2* __restrict__ idx = a.idx;
  // operand loads are buffer loads (see gemm_bs.hip): this row tile of the
  // activations and the packed weight blocks as scalar resources, one 32-bit
  // offset register per lane, the slab / block part of the address scalar
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)a.X + (size_t)rt * a.S_in * 8192), 0, a.S_in * 8192, 0x00020000);
  const __amdgpu_buffer_rsrc_t wres =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.blocks, 0, a.n_blocks * 16384, 0x00020000);
  const int xlo = lane * 16;
  typedef float v4f_t __attribute__((ext_vector_type(4)));
  auto bufld = [&](const __amdgpu_buffer_rsrc_t& r, int voff, int soff) {
    const v4f_t v = __builtin_bit_cast(v4f_t, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
    return make_float4(v.x, v.y, v.z, v.w);
  };
  const float al = a.alpha;
  const int spj = a.spj_in;

  if constexpr (PRO == PRO_BNACT) {
    for (int c = threadIdx.x; c < a.pro_F; c += 256) {
      dyn[c] = a.pro_scale[c];
      dyn[a.pro_F + c] = a.pro_shift[c];
    }
  }
  if constexpr (EPI == EPI_BNBACK) {
    const int ch = (so % (a.epi_F / kSlab)) * kSlab + lane;
    const float* src = w == 0 ? a.epi_scale : w == 1 ? a.epi_shift : w == 2 ? a.epi_mean : a.epi_rstd;
    tab[threadIdx.x] = src[ch];
  }
  if constexpr (PRO == PRO_BNACT || EPI == EPI_BNBACK) __syncthreads();

  auto load = [&](SlabRegs& s, int e) {
    const int2 ix = idx[e];  // wave-uniform
    const int si = __builtin_amdgcn_readfirstlane(ix.x), blk = __builtin_amdgcn_readfirstlane(ix.y);
#pragma unroll
    for (int g = 0; g < 8; ++g) s.x[g] = bufld(xres, xlo + (g & 3) * 1024, si * 8192 + (g >> 2) * 4096);
#pragma unroll
    for (int g = 0; g < 16; ++g) s.w[g] = bufld(wres, xlo + (g & 3) * 1024, blk * 16384 + (g >> 2) * 4096);
    return si;
  };
  f32x16 acc0, acc1;
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; }
  auto compute = [&](SlabRegs& s, int si) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      float4 xv = s.x[g];
      if constexpr (PRO == PRO_BNACT) {
        const int c_ = (si % spj) * kSlab + 8 * g + 4 * h;
        xv = bnact4(xv, *(const float4*)(dyn + c_), *(const float4*)(dyn + a.pro_F + c_), al);
      }
      const float4 w0 = s.w[2 * g], w1 = s.w[2 * g + 1];
      acc0 = MFMA32(w0.x, xv.x, acc0);
      acc1 = MFMA32(w1.x, xv.x, acc1);
      acc0 = MFMA32(w0.y, xv.y, acc0);
      acc1 = MFMA32(w1.y, xv.y, acc1);
      acc0 = MFMA32(w0.z, xv.z, acc0);
      acc1 = MFMA32(w1.z, xv.z, acc1);
      acc0 = MFMA32(w0.w, xv.w, acc0);
      acc1 = MFMA32(w1.w, xv.w, acc1);
    }
  };
  // wave w: entries beg + w, beg + w + 4, ... (two register sets, one slab ahead)
  SlabRegs sa, sb;
  int e = beg + w;
  if (e < end) {
    int sia = load(sa, e), sib = 0;
    for (;;) {
      const bool n1 = e + 4 < end;
      if (n1) sib = load(sb, e + 4);
      compute(sa, sia);
      if (!n1) break;
      const bool n2 = e + 8 < end;
      if (n2) sia = load(sa, e + 8);
      compute(sb, sib);
      if (!n2) break;
      e += 8;
    }
  }

  // ---- the four partial sums, added in wave order by wave 0 ----
  const int S_out = a.S_out;
  const int tbase = (rt * S_out + so) * 512 + lane;  // float4 index of chunk 0 of the output tile
  float v[32];
#pragma unroll
  for (int k = 0; k < 16; ++k) { v[k] = acc0[k]; v[16 + k] = acc1[k]; }
  if (w > 0) {
    float4* r4 = (float4*)(red + (w - 1) * 2048) + lane;
#pragma unroll
    for (int q = 0; q < 8; ++q) r4[q * 64] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
  __syncthreads();
  if (w > 0) return;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float4* r4 = (const float4*)(red + i * 2048) + lane;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 p = r4[q * 64];
      v[4 * q] += p.x; v[4 * q + 1] += p.y; v[4 * q + 2] += p.z; v[4 * q + 3] += p.w;
    }
  }
  // accumulator value i of lane half h is feature acc_feature(i, h); the float4
  // chunk q' = 0..7 of the output tile holds features 8q' + 4h .. +3, i.e.
  // v[4q..] for q' = q (acc0: features 0..31) and v[16 + 4q..] for q' = 4 + q
  float4 zq[8];
  if constexpr (EPI == EPI_BNBACK) {
    const float4* Z4 = (const float4*)a.epi_z + tbase;
#pragma unroll
    for (int q = 0; q < 8; ++q) zq[q] = Z4[q * 64];
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float4 add = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.bias) add = *(const float4*)(a.bias + so * kSlab + 8 * q + 4 * h);
    if (a.addsrc) {
      const float4 r = ((const float4*)a.addsrc)[tbase + q * 64];
      add.x += r.x; add.y += r.y; add.z += r.z; add.w += r.w;
    }
    // gemm_bs_kernel seeds the accumulators with the bias and adds the residual
    // last; adding both last differs in rounding only
    v[4 * q] += add.x; v[4 * q + 1] += add.y; v[4 * q + 2] += add.z; v[4 * q + 3] += add.w;
  }
  {
    float4* Y = (float4*)a.Y;
#pragma unroll
    for (int q = 0; q < 8; ++q) Y[tbase + q * 64] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
  if constexpr (EPI == EPI_NONE) return;

  // ---- BN partials of this 32-row tile (wave 0 alone: its LDS operations run
  // in issue order, no barrier) ----
  float* tr = red;  // 8 KB transposition buffer (the partial sums have been read)
  const int c = lane, cg = c >> 3, chh = (c >> 2) & 1, cs = c & 3;
  const int n = min(kRT, a.B - rt * kRT);  // valid rows of the tile
  float2* stat = a.stat + (size_t)rt * (S_out * kSlab) + so * kSlab + c;
  auto put = [&](int q, float x0, float x1, float x2, float x3) {
    const int pos = lane ^ (2 * q + h);
    *(float4*)(tr + (q * 64 + pos) * 4) = make_float4(x0, x1, x2, x3);
  };
  auto get = [&](int r) {  // value of row r of column c
    const int l = r + 32 * chh;
    return tr[(cg * 64 + (l ^ (2 * cg + chh))) * 4 + cs];
  };
  auto colsum = [&]() {
    float s = 0.f;
    for (int r = 0; r < n; ++r) s += get(r);
    return s;
  };
  if constexpr (EPI == EPI_BNFWD) {
#pragma unroll
    for (int q = 0; q < 8; ++q) put(q, v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    __builtin_amdgcn_wave_barrier();
    const float sum = colsum();
    const float mean = sum / (float)n;
    float m2 = 0.f;
    for (int r = 0; r < n; ++r) {
      const float d = get(r) - mean;
      m2 = fmaf(d, d, m2);
    }
    *stat = make_float2(sum, m2);
  } else {
    // EPI_BNBACK: du = dh * leaky'(u(z)), zhat = (z - mean) * rstd of the layer
    // below; the partials are (sum du, sum du * zhat)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 z4 = zq[q];
      const int ch = 8 * q + 4 * h;
      const float4 sc = *(const float4*)(tab + ch), sh = *(const float4*)(tab + 64 + ch);
      v[4 * q + 0] = fmaf(z4.x, sc.x, sh.x) > 0.f ? v[4 * q + 0] : v[4 * q + 0] * al;
      v[4 * q + 1] = fmaf(z4.y, sc.y, sh.y) > 0.f ? v[4 * q + 1] : v[4 * q + 1] * al;
      v[4 * q + 2] = fmaf(z4.z, sc.z, sh.z) > 0.f ? v[4 * q + 2] : v[4 * q + 2] * al;
      v[4 * q + 3] = fmaf(z4.w, sc.w, sh.w) > 0.f ? v[4 * q + 3] : v[4 * q + 3] * al;
      put(q, v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
    __builtin_amdgcn_wave_barrier();
    const float P = colsum();
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 z4 = zq[q];
      const int ch = 8 * q + 4 * h;
      const float4 mu = *(const float4*)(tab + 128 + ch), rs = *(const float4*)(tab + 192 + ch);
      put(q, v[4 * q] * ((z4.x - mu.x) * rs.x), v[4 * q + 1] * ((z4.y - mu.y) * rs.y),
          v[4 * q + 2] * ((z4.z - mu.z) * rs.z), v[4 * q + 3] * ((z4.w - mu.w) * rs.w));
    }
    __builtin_amdgcn_wave_barrier();
    const float Q = colsum();
    *stat = make_float2(P, Q);
  }
}

// Same arguments as launch_gemm_bs; a.stat receives one partial per ROW TILE
// (32 rows).  No dropout variant of the BN-backward epilogue (the caller uses
// gemm_bs_kernel then).
void launch_gemm_bs_small(const GemmArgs& a, hipStream_t s) {
  const int grid = a.n_rt * a.n_out_slabs;
  const size_t dyn = a.pro_mode == PRO_BNACT ? 2 * (size_t)a.pro_F * sizeof(float) : 0;
#define LAUNCH(P, E) hipLaunchKernelGGL((gemm_bs_small_kernel<P, E>), dim3(grid), dim3(256), dyn, s, a)
  if (a.pro_mode == PRO_BNACT) {
    if (a.epi_mode == EPI_BNFWD) LAUNCH(PRO_BNACT, EPI_BNFWD);
    else LAUNCH(PRO_BNACT, EPI_NONE);
  } else {
    if (a.epi_mode == EPI_BNFWD) LAUNCH(PRO_RAW, EPI_BNFWD);
    else if (a.epi_mode == EPI_BNBACK) LAUNCH(PRO_RAW, EPI_BNBACK);
    else LAUNCH(PRO_RAW, EPI_NONE);
  }
#undef LAUNCH
}

}  // namespace lcn
