// Weight-gradient GEMM, FOUR blocks of one output slab per workgroup (gfx950).
//
// Same contract as gemm_dw_kernel (kernels_gemm.hip): dW_e(si, so) = A[:, si]^T .
// dZ[:, so] over a workgroup's items of the batch, one partial slab per block
// and slot.  Here a group is four blocks (si_0..si_3, so) and wave w owns block
// w whole (64 x 64: four 32x32 accumulators), so the staged D slab -- its two
// loads per thread, its BN-backward rebuild, its transposed scatter -- serves
// four blocks instead of two, a 32-row stage holds 64 MFMAs per wave between
// its two barriers instead of 32 (four fragment reads per 16 MFMAs), and an
// output slab's dh / z rows are read by half as many workgroups.  146-168
// VGPRs, 49 KB of LDS: three workgroups per CU.
//
// Runs the hidden layers where every output slab holds a multiple of four
// blocks (four slabs per joint: the cfg4 shape, 68 blocks a slab; 16 384 rows:
// 5.34-5.48 -> 5.20 ms a launch, the step 180.2-184.2 -> 177.9-178.0 ms on one
// box).  Measured in gemm_bench at cfg3 (B = 65 536, knn 3; raw / BN-backward D /
// + BN-apply A, % of the fp32 MFMA peak): the 37 complete quads (148 of 175
// blocks) 78.2 / 74.2 / 71.6 % for the kernel alone against 79.3 / 71.3 / 68.5 %
// for the two-block kernel over all blocks with its partial reduce (2 %).  With
// one slab per joint the output slabs hold 5..17 blocks, and no way of running
// the 27 blocks left over (a launch of their own; a sub-tile wave map for groups
// of 1..3 in the same launch at three workgroups per CU; a sub-tile map for every
// group size) kept more than 2 % of that over all blocks, so there the two-block
// kernel stays.
#include "gemm_common.h"

namespace lcn {

constexpr int kDw4Ld = 36;

template <bool PRO, bool DBB, bool DROP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void gemm_dw4_kernel(GemmDwArgs a) {
  __shared__ __attribute__((aligned(16))) float Ds[64 * kDw4Ld];      // [q][row]
  __shared__ __attribute__((aligned(16))) float As[4][64 * kDw4Ld];   // [p][row] per block
  // channel constants: A (sc, sh) of the four input slabs; D sc, sh, c1, c2, c3, c1 * alpha
  __shared__ __attribute__((aligned(16))) float tab[14 * 64];
  const int4 wgm = a.wgmap[blockIdx.x];
  const int gi = __builtin_amdgcn_readfirstlane(wgm.x), slot = __builtin_amdgcn_readfirstlane(wgm.y);
  const int item0 = __builtin_amdgcn_readfirstlane(wgm.z), n_it = __builtin_amdgcn_readfirstlane(wgm.w);
  if (gi < 0) return;  // padding of the grid (uniform per workgroup)
  // group: (so, 4, rank, count), (b0, b1, b2, b3)
  const int4 grp = a.groups[2 * gi], gb = a.groups[2 * gi + 1];
  const DwPlan pl = a.plan;
  const int so = __builtin_amdgcn_readfirstlane(grp.x);
  const int bq[4] = {__builtin_amdgcn_readfirstlane(gb.x), __builtin_amdgcn_readfirstlane(gb.y),
                     __builtin_amdgcn_readfirstlane(gb.z), __builtin_amdgcn_readfirstlane(gb.w)};
  int si[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) si[k] = __builtin_amdgcn_readfirstlane(a.blk[bq[k]].x);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(w);
  const int lr = lane & 31, h = lane >> 5;
  const int wrank = __builtin_amdgcn_readfirstlane(grp.z), wcount = __builtin_amdgcn_readfirstlane(grp.w);
  const bool may_write = DBB && a.dz_out != nullptr;
  const int R = pl.item_rows, istride = pl.stride;

  {
    const int c = t & 63, k = t >> 6;  // 4 x 64 entries per pass
    if constexpr (PRO) {
      const int chk = ((k == 0 ? si[0] : k == 1 ? si[1] : k == 2 ? si[2] : si[3]) % a.spj_a) * kSlab + c;
      // leaky(u) = u' + ((1 - alpha) / (1 + alpha)) |u'| for u' = u (1 + alpha) / 2: tables pre-scaled
      tab[128 * k + c] = 0.5f * (1.f + a.alpha) * a.pro_scale[chk];
      tab[128 * k + 64 + c] = 0.5f * (1.f + a.alpha) * a.pro_shift[chk];
    }
    if constexpr (DBB) {
      const int ch = (so % a.spj_d) * kSlab + c, F = a.d_F;
      tab[512 + t] = k == 0 ? a.d_scale[ch] : k == 1 ? a.d_shift[ch] : k == 2 ? a.d_c123[ch] : a.d_c123[F + ch];
      if (k == 0) tab[768 + c] = a.d_c123[2 * F + ch];
      if (k == 1) tab[832 + c] = a.d_c123[ch] * a.alpha;
    }
  }

  f32x16 acc0, acc1, acc2, acc3;  // this wave's block: (rows 0..31 | 32..63) x (columns 0..31 | 32..63)
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; acc2[k] = 0.f; acc3[k] = 0.f; }
  [[maybe_unused]] Dropout dr{};
  if constexpr (DROP) dr = drop_resolve(a.d_drop);

  // this thread's staging slots: the same four features f0 .. f0 + 3 of two
  // rows, sr and sr + 16, of the stage's row tile
  const int S_a = a.S_a, S_d = a.S_d;
  const int sr = t & 15;
  const int c40 = (t >> 5) * 64 + ((t >> 4) & 1) * 32 + sr, c41 = c40 + 16;
  const int f0 = 8 * (t >> 5) + 4 * ((t >> 4) & 1);
  float4 ra[4][2], rd0, rd1, rz0, rz1;
  const int ntile = (a.B + kRT - 1) / kRT;
  const __amdgpu_buffer_rsrc_t ares =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.A, 0, (unsigned)ntile * S_a * 8192u, 0x00020000);
  const __amdgpu_buffer_rsrc_t dres =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.D, 0, (unsigned)ntile * S_d * 8192u, 0x00020000);
  const __amdgpu_buffer_rsrc_t zres =
      __builtin_amdgcn_make_buffer_rsrc((void*)(DBB ? a.d_z : a.D), 0, (unsigned)ntile * S_d * 8192u, 0x00020000);
  typedef float v4f_t __attribute__((ext_vector_type(4)));
#define DW_BUFLD(RES, VOFF, SOFF)                                                      \
  ({                                                                                   \
    const v4f_t v_ = __builtin_bit_cast(v4f_t, __builtin_amdgcn_raw_buffer_load_b128((RES), (VOFF), (SOFF), 0)); \
    make_float4(v_.x, v_.y, v_.z, v_.w);                                               \
  })
  const int v40 = c40 * 16, v41 = c41 * 16;
#define DW_GLOAD(BASE)                                                     \
  {                                                                        \
    const int t_ = (BASE) / kRT;                                           \
    const int od = (int)((unsigned)(t_ * S_d + so) * 8192u);               \
    _Pragma("unroll") for (int k = 0; k < 4; ++k) {                        \
      {                                                                    \
        const int oa = (int)((unsigned)(t_ * S_a + si[k]) * 8192u);        \
        ra[k][0] = DW_BUFLD(ares, v40, oa);                                \
        ra[k][1] = DW_BUFLD(ares, v41, oa);                                \
      }                                                                    \
    }                                                                      \
    rd0 = DW_BUFLD(dres, v40, od);                                         \
    rd1 = DW_BUFLD(dres, v41, od);                                         \
    if constexpr (DBB) {                                                   \
      rz0 = DW_BUFLD(zres, v40, od);                                       \
      rz1 = DW_BUFLD(zres, v41, od);                                       \
    }                                                                      \
  }
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
    __syncthreads();  // previous stage's fragment reads are done (and the tables written)
    const bool v0 = base + sr < r1, v1 = base + sr + 16 < r1;
    // transposed scatter: feature -> LDS row, batch row -> column
#define DW_PUT(P, F4, OFF)             \
  P[(OFF)] = (F4).x;                   \
  P[(OFF) + kDw4Ld] = (F4).y;          \
  P[(OFF) + 2 * kDw4Ld] = (F4).z;      \
  P[(OFF) + 3 * kDw4Ld] = (F4).w;
    const int o0 = f0 * kDw4Ld + sr, o1 = o0 + 16;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);  // rows past the item's end contribute nothing
    // the D slab first (its coefficients are dead before the A slabs' tables are read), then block by
    // block: no instance spills (all four blocks transformed ahead of the scatter: 28 registers spilled)
    if constexpr (DBB) {
      BnBackCoef cf;
      cf.sc = *(const float4*)(tab + 512 + f0); cf.sh = *(const float4*)(tab + 576 + f0);
      cf.c1 = *(const float4*)(tab + 640 + f0); cf.c2 = *(const float4*)(tab + 704 + f0);
      cf.c3 = *(const float4*)(tab + 768 + f0);
      const float4 c1a = *(const float4*)(tab + 832 + f0);
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
        const size_t t_ = base / kRT;
        if (v0) o[(t_ * S_d + so) * 512 + c40] = rd0;
        if (v1) o[(t_ * S_d + so) * 512 + c41] = rd1;
      }
    }
    if (!v0) rd0 = z4;
    if (!v1) rd1 = z4;
    DW_PUT(Ds, rd0, o0) DW_PUT(Ds, rd1, o1)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (PRO) {
        const float ba = (1.f - a.alpha) / (1.f + a.alpha);
        const float4 sc = *(const float4*)(tab + 128 * k + f0), sh = *(const float4*)(tab + 128 * k + 64 + f0);
        ra[k][0] = bnact4_scaled(ra[k][0], sc, sh, ba);
        ra[k][1] = bnact4_scaled(ra[k][1], sc, sh, ba);
      }
      if (!v0) ra[k][0] = z4;
      if (!v1) ra[k][1] = z4;
      DW_PUT(As[k], ra[k][0], o0) DW_PUT(As[k], ra[k][1], o1)
    }
#undef DW_PUT
    // the next stage's loads go out before the barrier (its wait hides part of
    // their latency), and the MFMA phase runs at raised wave priority
    if (nmore) DW_GLOAD(nbase);
    __syncthreads();
    __builtin_amdgcn_s_setprio(1);
    {
      const float* A0 = As[wv] + lr * kDw4Ld + 4 * h;
      const float* A1 = As[wv] + (32 + lr) * kDw4Ld + 4 * h;
      const float* D0 = Ds + lr * kDw4Ld + 4 * h;
      const float* D1 = Ds + (32 + lr) * kDw4Ld + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 a0 = *(const float4*)(A0 + 8 * g), a1 = *(const float4*)(A1 + 8 * g);
        const float4 d0 = *(const float4*)(D0 + 8 * g), d1 = *(const float4*)(D1 + 8 * g);
#define DW4_K(C)                                                                \
        acc0 = MFMA32(a0.C, d0.C, acc0); acc1 = MFMA32(a0.C, d1.C, acc1);       \
        acc2 = MFMA32(a1.C, d0.C, acc2); acc3 = MFMA32(a1.C, d1.C, acc3);
        DW4_K(x) DW4_K(y) DW4_K(z) DW4_K(w)
#undef DW4_K
      }
    }
    __builtin_amdgcn_s_setprio(0);
    base = nbase;
    it = nit;
    item = nitem;
    iend = nend;
    more = nmore;
  }
#undef DW_GLOAD
#undef DW_BUFLD
  {  // this slot's partial of this wave's block
    const int myblk = wv == 0 ? bq[0] : wv == 1 ? bq[1] : wv == 2 ? bq[2] : bq[3];
    float* out = a.part + ((size_t)slot * a.nblk + myblk) * 4096;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int p = (k & 3) + 8 * (k >> 2) + 4 * h;
      out[p * 64 + lr] = acc0[k];
      out[p * 64 + 32 + lr] = acc1[k];
      out[(32 + p) * 64 + lr] = acc2[k];
      out[(32 + p) * 64 + 32 + lr] = acc3[k];
    }
  }
}

int gemm_dw4_resident_slots() {
  int dev = 0, per_cu = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm_dw4_kernel<true, true, false>, 256, 0) != hipSuccess)
    return 0;
  return per_cu * prop.multiProcessorCount;
}

void launch_gemm_dw4(const GemmDwArgs& a, hipStream_t s) {
  const int grid = a.n_wg;
  const bool pro = a.pro_scale != nullptr, dbb = a.d_bnback != 0;
  const bool drop = dbb && a.d_drop.rate > 0.f;
  if (pro && drop)
    hipLaunchKernelGGL((gemm_dw4_kernel<true, true, true>), dim3(grid), dim3(256), 0, s, a);
  else if (drop)
    hipLaunchKernelGGL((gemm_dw4_kernel<false, true, true>), dim3(grid), dim3(256), 0, s, a);
  else if (pro && dbb)
    hipLaunchKernelGGL((gemm_dw4_kernel<true, true, false>), dim3(grid), dim3(256), 0, s, a);
  else if (pro)
    hipLaunchKernelGGL((gemm_dw4_kernel<true, false, false>), dim3(grid), dim3(256), 0, s, a);
  else if (dbb)
    hipLaunchKernelGGL((gemm_dw4_kernel<false, true, false>), dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_dw4_kernel<false, false, false>), dim3(grid), dim3(256), 0, s, a);
}

}  // namespace lcn
