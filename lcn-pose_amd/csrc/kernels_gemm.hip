// Weight-gradient GEMM of the LCN layers (gfx950): for every present 64x64
// block (si, so), dW_e = A[:, si-slab]^T . dZ[:, so-slab] summed over the
// batch (the dW half of the autodiff of models_att.py:662, :692, and of the
// thin lift / output layers).  The batch is split into chunks; each chunk
// writes a partial slab that dw_reduce sums in a fixed order (deterministic,
// no atomics).
#include <cstdlib>

#include "gemm_common.h"

namespace lcn {

// One workgroup = a group of up to two 64x64 blocks (si0, so), (si1, so) x
// one slot of the batch (DwPlan: a strided set of row items); waves (bi, hp) = (w >> 1, w & 1) compute rows 32hp..+31 of
// block bi against all 64 columns (two 32x32 accumulators), so the staged D
// slab -- and its BN-backward rebuild -- serves both blocks.  A group of one
// block (the last of an output slab with an odd number of blocks) splits the
// block four ways instead, wave (qh, hp) = (w >> 1, w & 1) computing rows
// 32hp..+31 x columns 32qh..+31 in one accumulator: half the MFMAs per stage,
// no idle wave.  One 32-row tile per LDS stage.  The slots are placed by XCD
// (make_dw_wgmap) so the groups that read the same rows at the same time share
// the activation tiles through that XCD's L2.
//
// Staging: every thread loads 2 float4 of each operand's 8 KB row-tile slab
// (coalesced 1 KB chunks), applies the operand transform (channel constants
// from small LDS tables), and scatters them transposed into LDS as
// [feature][row] with row stride 36 floats: the ds_write_b32 scatter and the
// ds_read_b128 fragment reads (lane l reads feature l & 31, rows 8g + 4h ..
// +3) are both bank-conflict free.  The MFMA runs over the batch: k = row.
//
// PRO: the A operand gets BN apply + LeakyReLU (A = z of the layer below the
// block's inner layer); DBB: the D operand is dz rebuilt from (dh, z) by the
// BN + LeakyReLU backward, dz = c1 du + c2 + c3 z; the groups of an output slab
// take turns storing that dz (dz_out) for the backward-data GEMM that follows, so dz
// costs one write and no separate elementwise pass.
constexpr int kDwLd = 36;

template <bool PRO, bool DBB, bool DROP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void gemm_dw_kernel(GemmDwArgs a) {
  __shared__ __attribute__((aligned(16))) float Ds[64 * kDwLd];      // [q][row]
  __shared__ __attribute__((aligned(16))) float As[2][64 * kDwLd];   // [p][row] per block
  // channel constants: A sc, sh of si0; A sc, sh of si1 (both times (1 + alpha) / 2);
  // D sc, sh, c1, c2, c3, c1 * alpha
  __shared__ __attribute__((aligned(16))) float tab[10 * 64];
#ifdef EXP_CLOCK
  const uint64_t ck0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  // Work map (DwPlan, make_dw_wgmap): this workgroup's group of blocks, its
  // partial slot, and its items item0, item0 + stride, ... (n_it of them), all
  // accumulated in registers.
  const DwPlan pl = a.plan;
  const int4 wgm = a.wgmap[blockIdx.x];
  const int gi = __builtin_amdgcn_readfirstlane(wgm.x), slot = __builtin_amdgcn_readfirstlane(wgm.y);
  const int item0 = __builtin_amdgcn_readfirstlane(wgm.z), n_it = __builtin_amdgcn_readfirstlane(wgm.w);
  if (gi < 0) return;  // padding of the grid (uniform per workgroup)
  const int4 grp = a.groups[gi];
  // workgroup-uniform: kept in scalar registers (they form the scalar offsets of the operand loads)
  const int so = __builtin_amdgcn_readfirstlane(grp.x), b0 = __builtin_amdgcn_readfirstlane(grp.y),
            b1 = __builtin_amdgcn_readfirstlane(grp.z);
  const bool two = b1 >= 0;
  const int si0 = __builtin_amdgcn_readfirstlane(a.blk[b0].x);
  const int si1 = two ? __builtin_amdgcn_readfirstlane(a.blk[b1].x) : si0;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int lr = lane & 31, h = lane >> 5;
  const int bi = w >> 1, hp = w & 1;
  // the groups of an output slab all rebuild the same dz: item i is stored by the
  // group of rank i % count, so the stores are spread evenly over them
  const int wrank = __builtin_amdgcn_readfirstlane(grp.w) & 255, wcount = __builtin_amdgcn_readfirstlane(grp.w) >> 8;
  const bool may_write = DBB && a.dz_out != nullptr;
  const int R = pl.item_rows, istride = pl.stride;

  {
    const int c = t & 63, k = t >> 6;  // 4 x 64 entries per pass
    if constexpr (PRO) {
      // leaky(u) = max(u, alpha u) = a u + b |u| with a = (1 + alpha) / 2, b = (1 - alpha) / 2: with the
      // tables scaled by a, the operand is u' + (b / a) |u'|, two operations an element instead of three
      // (within 2 ulp of the max form; the operand of the weight gradient only)
      const int ch0 = (si0 % a.spj_a) * kSlab + c, ch1 = (si1 % a.spj_a) * kSlab + c;
      tab[t] = 0.5f * (1.f + a.alpha) *
               (k == 0 ? a.pro_scale[ch0] : k == 1 ? a.pro_shift[ch0] : k == 2 ? a.pro_scale[ch1] : a.pro_shift[ch1]);
    }
    if constexpr (DBB) {
      const int ch = (so % a.spj_d) * kSlab + c, F = a.d_F;
      tab[256 + t] = k == 0 ? a.d_scale[ch] : k == 1 ? a.d_shift[ch] : k == 2 ? a.d_c123[ch] : a.d_c123[F + ch];
      if (k == 0) tab[512 + c] = a.d_c123[2 * F + ch];
      if (k == 1) tab[576 + c] = a.d_c123[ch] * a.alpha;
    }
  }

  f32x16 acc0, acc1;
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; }
  [[maybe_unused]] Dropout dr{};
  if constexpr (DROP) dr = drop_resolve(a.d_drop);

  // this thread's staging slots: the same four features f0 .. f0 + 3 of two
  // rows, sr and sr + 16, of the stage's row tile (float4 c40, c40 + 16 of the
  // slab: chunk g = t >> 5, lane half (t >> 4) & 1) -- one set of channel
  // constants serves both
  const int S_a = a.S_a, S_d = a.S_d;
  const int sr = t & 15;
  const int c40 = (t >> 5) * 64 + ((t >> 4) & 1) * 32 + sr, c41 = c40 + 16;
  const int f0 = 8 * (t >> 5) + 4 * ((t >> 4) & 1);
  float4 ra0, ra1, rb0, rb1, rd0, rd1, rz0, rz1;
#define DW_IX(RT, S, SL, C4) (((size_t)(RT) * (S) + (SL)) * 512 + (C4))
#ifdef EXP_DW_HOT  // diagnostic build: every stage reads one of four row tiles (operands stay in L2)
#define DW_TILE(BASE) (((BASE) / kRT) & 3)
  const int tile0 = 0;
#else
#define DW_TILE(BASE) ((BASE) / kRT)
  const int tile0 = 0;
#endif
  // Operand loads are buffer loads (gemm_bs.hip): one resource per operand over
  // all its row tiles (< 4 GB: checked by the launcher), the (tile, slab) part
  // of the address in scalar registers, this thread's two float4 slots as
  // constant lane offsets.
#ifdef EXP_DW_HOT
  const int ntile = 4;
#else
  const int ntile = (a.B + kRT - 1) / kRT;
#endif
  const __amdgpu_buffer_rsrc_t ares = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)a.A + (size_t)tile0 * S_a * 8192), 0, (unsigned)ntile * S_a * 8192u, 0x00020000);
  const __amdgpu_buffer_rsrc_t dres = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)a.D + (size_t)tile0 * S_d * 8192), 0, (unsigned)ntile * S_d * 8192u, 0x00020000);
  const __amdgpu_buffer_rsrc_t zres = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)(DBB ? a.d_z : a.D) + (size_t)tile0 * S_d * 8192), 0, (unsigned)ntile * S_d * 8192u, 0x00020000);
  typedef float v4f_t __attribute__((ext_vector_type(4)));
#define DW_BUFLDX(RES, VOFF, SOFF, AUX)                                                \
  ({                                                                                   \
    const v4f_t v_ = __builtin_bit_cast(v4f_t, __builtin_amdgcn_raw_buffer_load_b128((RES), (VOFF), (SOFF), (AUX))); \
    make_float4(v_.x, v_.y, v_.z, v_.w);                                               \
  })
  // diagnostic builds: cache policy bits (2 = nt) of the A / D,z loads
#ifndef EXP_DW_AUX_A
#define EXP_DW_AUX_A 0
#endif
#ifndef EXP_DW_AUX_D
#define EXP_DW_AUX_D 0
#endif
#define DW_BUFLD(RES, VOFF, SOFF) DW_BUFLDX(RES, VOFF, SOFF, EXP_DW_AUX_A)
#define DW_BUFLDD(RES, VOFF, SOFF) DW_BUFLDX(RES, VOFF, SOFF, EXP_DW_AUX_D)
  const int v40 = c40 * 16, v41 = c41 * 16;
#define DW_GLOAD(BASE)                                                     \
  {                                                                        \
    const int t_ = DW_TILE(BASE) - tile0;                                  \
    const int oa0 = (int)((unsigned)(t_ * S_a + si0) * 8192u), od = (int)((unsigned)(t_ * S_d + so) * 8192u); \
    ra0 = DW_BUFLD(ares, v40, oa0);                                        \
    ra1 = DW_BUFLD(ares, v41, oa0);                                        \
    if (two) {                                                             \
      const int oa1 = (int)((unsigned)(t_ * S_a + si1) * 8192u);           \
      rb0 = DW_BUFLD(ares, v40, oa1);                                      \
      rb1 = DW_BUFLD(ares, v41, oa1);                                      \
    }                                                                      \
    rd0 = DW_BUFLDD(dres, v40, od);                                        \
    rd1 = DW_BUFLDD(dres, v41, od);                                        \
    if constexpr (DBB) {                                                   \
      rz0 = DW_BUFLDD(zres, v40, od);                                      \
      rz1 = DW_BUFLDD(zres, v41, od);                                      \
    }                                                                      \
  }
  // stages of this workgroup: its items, 32 rows a stage; the next stage's rows
  // are known one stage ahead (its loads go out early)
  int it = 0, item = item0, base = item0 * R, iend = min(a.B, base + R);
  bool more = n_it > 0 && base < a.B;
  if (more) DW_GLOAD(base);
  while (more) {
    int nbase = base + kRT, nit = it, nitem = item, nend = iend;
    if (nbase >= iend) {
      nit = it + 1;
      nitem = item + istride;
      nbase = nitem * R;
      nend = min(a.B, nbase + R);
    }
    const bool nmore = nit < n_it && nbase < a.B;
    const int r1 = iend;
    const bool writer = may_write && item % wcount == wrank;
#ifndef EXP_DW_NOBAR1
    __syncthreads();  // previous stage's fragment reads are done (and the tables written)
#endif
    const bool v0 = base + sr < r1, v1 = base + sr + 16 < r1;
#ifndef EXP_DW_NOSTAGE  // diagnostic build without the staging phase (loads, transforms, scatter)
    if constexpr (PRO) {
      const float ba = (1.f - a.alpha) / (1.f + a.alpha);
      const float4 sc0 = *(const float4*)(tab + f0), sh0 = *(const float4*)(tab + 64 + f0);
      ra0 = bnact4_scaled(ra0, sc0, sh0, ba);
      ra1 = bnact4_scaled(ra1, sc0, sh0, ba);
      if (two) {
        const float4 sc1 = *(const float4*)(tab + 128 + f0), sh1 = *(const float4*)(tab + 192 + f0);
        rb0 = bnact4_scaled(rb0, sc1, sh1, ba);
        rb1 = bnact4_scaled(rb1, sc1, sh1, ba);
      }
    }
    if constexpr (DBB) {
      BnBackCoef cf;
      cf.sc = *(const float4*)(tab + 256 + f0); cf.sh = *(const float4*)(tab + 320 + f0);
      cf.c1 = *(const float4*)(tab + 384 + f0); cf.c2 = *(const float4*)(tab + 448 + f0);
      cf.c3 = *(const float4*)(tab + 512 + f0);
      const float4 c1a = *(const float4*)(tab + 576 + f0);
      if constexpr (DROP) {  // tf.nn.dropout's gradient: dh * mask * scale
        const int64_t row = base + sr;
        const int col = so * kSlab + f0;
        rd0.x = drop_apply(dr, row, col, rd0.x);
        rd0.y = drop_apply(dr, row, col + 1, rd0.y);
        rd0.z = drop_apply(dr, row, col + 2, rd0.z);
        rd0.w = drop_apply(dr, row, col + 3, rd0.w);
        rd1.x = drop_apply(dr, row + 16, col, rd1.x);
        rd1.y = drop_apply(dr, row + 16, col + 1, rd1.y);
        rd1.z = drop_apply(dr, row + 16, col + 2, rd1.z);
        rd1.w = drop_apply(dr, row + 16, col + 3, rd1.w);
      }
      rd0 = bnback4_sel(rd0, rz0, cf, c1a);
      rd1 = bnback4_sel(rd1, rz1, cf, c1a);
      if (writer) {
        float4* o = (float4*)a.dz_out;
        const int t_ = base / kRT;
        if (v0) o[DW_IX(t_, S_d, so, c40)] = rd0;
        if (v1) o[DW_IX(t_, S_d, so, c41)] = rd1;
      }
    }
    {  // rows past the chunk end contribute nothing
      const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!v0) { ra0 = z4; rb0 = z4; rd0 = z4; }
      if (!v1) { ra1 = z4; rb1 = z4; rd1 = z4; }
    }
    {
      // transposed scatter: feature -> LDS row, batch row -> column
#define DW_PUT(P, F4, OFF)             \
  P[(OFF)] = (F4).x;                   \
  P[(OFF) + kDwLd] = (F4).y;           \
  P[(OFF) + 2 * kDwLd] = (F4).z;       \
  P[(OFF) + 3 * kDwLd] = (F4).w;
      const int o0 = f0 * kDwLd + sr, o1 = o0 + 16;
      DW_PUT(As[0], ra0, o0) DW_PUT(As[0], ra1, o1)
      if (two) { DW_PUT(As[1], rb0, o0) DW_PUT(As[1], rb1, o1) }
      DW_PUT(Ds, rd0, o0) DW_PUT(Ds, rd1, o1)
#undef DW_PUT
    }
#endif
    // the next stage's loads go out before the barrier (its wait hides part of
    // their latency; 976 -> 914 us measured), and the MFMA phase runs at raised
    // wave priority so the other waves' staging does not starve it
    if (nmore) DW_GLOAD(nbase);
#ifndef EXP_DW_NOBAR2
    __syncthreads();
#endif
#if defined(EXP_DW_ROTPRIO)  // diagnostic: the priority of the MFMA phase rotates with the item, offset by dispatch layer
    switch (((blockIdx.x >> 8) + it) & 3) {
      case 0: __builtin_amdgcn_s_setprio(0); break;
      case 1: __builtin_amdgcn_s_setprio(1); break;
      case 2: __builtin_amdgcn_s_setprio(2); break;
      default: __builtin_amdgcn_s_setprio(3); break;
    }
#elif defined(EXP_DW_NOPRIO)   // diagnostic builds: no raised priority / a different level per workgroup
#elif defined(EXP_DW_PRIOWG)
    switch (blockIdx.x % 3) {
      case 0: __builtin_amdgcn_s_setprio(1); break;
      case 1: __builtin_amdgcn_s_setprio(2); break;
      default: __builtin_amdgcn_s_setprio(3); break;
    }
#else
    __builtin_amdgcn_s_setprio(1);
#endif
#ifndef EXP_DW_NOMFMA  // diagnostic build without the fragment reads and MFMAs
    if (two) {
      const float* Ap = As[bi] + (32 * hp + lr) * kDwLd + 4 * h;
      const float* D0 = Ds + lr * kDwLd + 4 * h;
      const float* D1 = Ds + (32 + lr) * kDwLd + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
#ifdef EXP_DW_FEWREADS  // diagnostic: one fragment set per stage instead of four
        const int go = 0;
#else
        const int go = 8 * g;
#endif
        const float4 av = *(const float4*)(Ap + go);
        const float4 d0 = *(const float4*)(D0 + go);
        const float4 d1 = *(const float4*)(D1 + go);
        acc0 = MFMA32(av.x, d0.x, acc0);
        acc1 = MFMA32(av.x, d1.x, acc1);
        acc0 = MFMA32(av.y, d0.y, acc0);
        acc1 = MFMA32(av.y, d1.y, acc1);
        acc0 = MFMA32(av.z, d0.z, acc0);
        acc1 = MFMA32(av.z, d1.z, acc1);
        acc0 = MFMA32(av.w, d0.w, acc0);
        acc1 = MFMA32(av.w, d1.w, acc1);
      }
    } else {  // one block: this wave's quarter (rows 32hp.., columns 32bi..)
      const float* Ap = As[0] + (32 * hp + lr) * kDwLd + 4 * h;
      const float* Dq = Ds + (32 * bi + lr) * kDwLd + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 av = *(const float4*)(Ap + 8 * g);
        const float4 dv = *(const float4*)(Dq + 8 * g);
        acc0 = MFMA32(av.x, dv.x, acc0);
        acc0 = MFMA32(av.y, dv.y, acc0);
        acc0 = MFMA32(av.z, dv.z, acc0);
        acc0 = MFMA32(av.w, dv.w, acc0);
      }
    }
#endif
    __builtin_amdgcn_s_setprio(0);
    base = nbase;
    it = nit;
    item = nitem;
    iend = nend;
    more = nmore;
  }
#undef DW_GLOAD
#undef DW_BUFLD
#undef DW_BUFLDD
#undef DW_BUFLDX
#undef DW_TILE
#undef DW_IX
#ifdef EXP_CLOCK
  if (threadIdx.x == 0 && a.clk) {
    const uint64_t ck1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    a.clk[4 * blockIdx.x] = ck1 - ck0;
    a.clk[4 * blockIdx.x + 1] = rt1 - rt0;
    a.clk[4 * blockIdx.x + 2] = rt0;
    a.clk[4 * blockIdx.x + 3] = rt1;
  }
#endif
  // this slot's partial of each block
  if (two) {
    float* out = a.part + ((size_t)slot * a.nblk + (bi ? b1 : b0)) * 4096;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int p = 32 * hp + (k & 3) + 8 * (k >> 2) + 4 * h;
      out[p * 64 + lr] = acc0[k];
      out[p * 64 + 32 + lr] = acc1[k];
    }
  } else {
    float* out = a.part + ((size_t)slot * a.nblk + b0) * 4096 + 32 * bi;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int p = 32 * hp + (k & 3) + 8 * (k >> 2) + 4 * h;
      out[p * 64 + lr] = acc0[k];
    }
  }
}

int gemm_dw_resident_slots() {
  // the instance the training step runs most (BN-apply A x BN-backward D); the
  // others need no more registers or LDS
  int dev = 0, per_cu = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm_dw_kernel<true, true, false>, 256, 0) != hipSuccess)
    return 0;
  return per_cu * prop.multiProcessorCount;
}

void launch_gemm_dw(const GemmDwArgs& a, hipStream_t s) {
  const int grid = a.n_wg;
#ifdef EXP_DW_LDSPAD  // diagnostic build: unused dynamic LDS per workgroup (bytes), to lower the residency
  const size_t pad = std::getenv("LCN_DW_LDSPAD") ? (size_t)std::atoi(std::getenv("LCN_DW_LDSPAD")) : 0;
#else
  const size_t pad = 0;
#endif
  const bool pro = a.pro_scale != nullptr, dbb = a.d_bnback != 0;
  // the dropout variants are separate instances: the mask hash costs registers
  const bool drop = dbb && a.d_drop.rate > 0.f;
  if (pro && drop)
    hipLaunchKernelGGL((gemm_dw_kernel<true, true, true>), dim3(grid), dim3(256), pad, s, a);
  else if (drop)
    hipLaunchKernelGGL((gemm_dw_kernel<false, true, true>), dim3(grid), dim3(256), pad, s, a);
  else if (pro && dbb)
    hipLaunchKernelGGL((gemm_dw_kernel<true, true, false>), dim3(grid), dim3(256), pad, s, a);
  else if (pro)
    hipLaunchKernelGGL((gemm_dw_kernel<true, false, false>), dim3(grid), dim3(256), pad, s, a);
  else if (dbb)
    hipLaunchKernelGGL((gemm_dw_kernel<false, true, false>), dim3(grid), dim3(256), pad, s, a);
  else
    hipLaunchKernelGGL((gemm_dw_kernel<false, false, false>), dim3(grid), dim3(256), pad, s, a);
}

// Sum the chunk partials of every block in a fixed order and scatter into the
// dense gradient dW[rows][ld]; rows / columns past (rows_valid, cols_valid)
// are the zero padding of the thin lift / output layers and are dropped.
// Each thread owns 4 adjacent columns (float4 loads) and keeps 8 chunk loads
// in flight; the additions stay in chunk order c = 0, 1, ... (deterministic,
// the same sums as a plain sequential loop).
__global__ __launch_bounds__(256) void dw_reduce_kernel(const float* __restrict__ part, int nchunks,
                                                        int nblk, const int2* __restrict__ blk,
                                                        float* __restrict__ dW, int ld,
                                                        int rows_valid, int cols_valid) {
  const int b = blockIdx.y;
  const int e = (blockIdx.x * 256 + threadIdx.x) * 4;  // 0..4092
  const int2 sb = blk[b];
  const int row = sb.x * kSlab + (e >> 6), col = sb.y * kSlab + (e & 63);
  if (row >= rows_valid || col >= cols_valid) return;
  const size_t stride4 = (size_t)nblk * 1024;
  const float4* p = (const float4*)(part + (size_t)b * 4096 + e);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  int c = 0;
  for (; c + 8 <= nchunks; c += 8) {
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p[(size_t)(c + k) * stride4];
#pragma unroll
    for (int k = 0; k < 8; ++k) { s.x += v[k].x; s.y += v[k].y; s.z += v[k].z; s.w += v[k].w; }
  }
  for (; c < nchunks; ++c) {
    const float4 v = p[(size_t)c * stride4];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  float* o = dW + (size_t)row * ld + col;
  const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (col + k < cols_valid) o[k] = sv[k];
}

void launch_dw_reduce(const float* part, int nchunks, int nblk, const int2* blk, float* dW, int ld,
                      int rows_valid, int cols_valid, hipStream_t s) {
  hipLaunchKernelGGL(dw_reduce_kernel, dim3(4, nblk), dim3(256), 0, s, part, nchunks, nblk, blk,
                     dW, ld, rows_valid, cols_valid);
}

}  // namespace lcn

