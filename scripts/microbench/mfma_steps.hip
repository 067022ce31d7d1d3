// Where the block-sparse GEMM's slab loop loses matrix-core time: a loop of 64
// v_mfma_f32_32x32x2_f32 per iteration (one input slab of gemm_bs_kernel), to
// which the loop's other ingredients are added one by one:
//   mode 0  MFMAs only (operands in registers)
//   mode 1  + a workgroup barrier per iteration
//   mode 2  + the 16 ds_read_b128 weight-fragment reads per iteration
//   mode 3  + 8 global_load_dwordx4 of activation fragments, one iteration ahead
//   mode 4  + the 4 LDS-DMA loads of the next weight block into the other buffer
//   mode 5  mode 4 with the two weight buffers as separate LDS objects and an
//           explicit vmcnt(0) ahead of the barrier (no compiler-inserted drain
//           before the first weight read)
//   mode 6  mode 5 with the 12 loads spread between the MFMAs (one load per
//           5 MFMAs) instead of issued in a burst
//   mode 7  mode 4 with buffer loads (scalar resource + one 32-bit offset
//           register per lane instead of a 64-bit address pair), activations
//           and LDS-DMA alike
//   mode 8  mode 7 with the loads spread between the MFMAs as in mode 6
//   mode 9  mode 7 with two accumulator pairs (two output slabs per wave): the
//           activation fragments are loaded on every other iteration only (both
//           output slabs multiply the same input slab), the weight DMA on every one
//   mode 10 mode 9's register shape (two accumulator pairs, alternating) with
//           the activation loads on every iteration: the control for mode 9
//   mode 11 the weight-gradient kernel's MFMA phase alone: per iteration two
//           barriers, 12 ds_read_b128 of transposed fragments (row stride 36
//           floats) and 32 MFMAs on two accumulators, no global loads
//   mode 12 mode 11 with one barrier per iteration; mode 13 with none
// 4 workgroups of 4 waves per CU as in the GEMM.  Results are meaningless; only
// the rate matters.
//   hipcc --offload-arch=gfx950 -O3 -o mfma_steps mfma_steps.hip && ./mfma_steps
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)
#define STEP(W0, W1, XV)                 \
  acc0 = MFMA32((W0).x, (XV).x, acc0);   \
  acc1 = MFMA32((W1).x, (XV).x, acc1);   \
  acc0 = MFMA32((W0).y, (XV).y, acc0);   \
  acc1 = MFMA32((W1).y, (XV).y, acc1);   \
  acc0 = MFMA32((W0).z, (XV).z, acc0);   \
  acc1 = MFMA32((W1).z, (XV).z, acc1);   \
  acc0 = MFMA32((W0).w, (XV).w, acc0);   \
  acc1 = MFMA32((W1).w, (XV).w, acc1);
#define GLDS(SRC, DST) \
  __builtin_amdgcn_global_load_lds((const void*)(SRC), (__attribute__((address_space(3))) void*)(DST), 16, 0, 0);

template <int MODE, int WPE = 4>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void loop_kernel(
    int iters, const float4* __restrict__ X, const float4* __restrict__ W, int n_tiles, float* out) {
  extern __shared__ __attribute__((aligned(16))) float4 Wl[];  // [2][1024]
  __shared__ __attribute__((aligned(16))) float4 Wa[(MODE == 5 || MODE == 6) ? 1024 : 1];
  __shared__ __attribute__((aligned(16))) float4 Wb[(MODE == 5 || MODE == 6) ? 1024 : 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f32x16 acc0, acc1, acc2, acc3;
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; acc2[k] = 0.f; acc3[k] = 0.f; }
  float4 xa[8], xb[8];
  for (int g = 0; g < 8; ++g) {
    xa[g] = make_float4(1e-3f * lane, 1e-3f * g, 1.f, 2.f);
    xb[g] = xa[g];
  }
  if (MODE == 5 || MODE == 6) {
    for (int i = threadIdx.x; i < 1024; i += 256) { Wa[i] = make_float4(1e-3f * i, 1.f, 2.f, 3.f); Wb[i] = Wa[i]; }
  } else {
    for (int i = threadIdx.x; i < 2048; i += 256) Wl[i] = make_float4(1e-3f * i, 1.f, 2.f, 3.f);
  }
  __syncthreads();
  // this wave's activation stream: tile (blockIdx.x * 4 + w + 13 * it) mod n_tiles, 8 KB each
  const float4* xw = X + lane;
  const int t0 = blockIdx.x * 4 + w;
  auto tile = [&](int it) { return (size_t)((t0 + 13 * it) % n_tiles) * 512; };
  auto utile = [&](int it) { return (unsigned)((t0 + 13 * it) % n_tiles) * 512u + (unsigned)lane; };
  if (MODE >= 3) {
#pragma unroll
    for (int g = 0; g < 8; ++g) xa[g] = xw[tile(0) + g * 64];
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, n_tiles * 8192, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, 175 * 16384, 0x00020000);
#define LOADXM(P, IT)                                                     \
  if ((MODE >= 7)) {                                                        \
    const int u_ = (int)(utile(IT) * 16u);                                \
    _Pragma("unroll") for (int g = 0; g < 8; ++g) {                       \
      const v4f v_ = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(xr, u_, g * 1024, 0)); \
      P[g] = make_float4(v_.x, v_.y, v_.z, v_.w);                         \
    }                                                                     \
  } else if (MODE >= 3) {                                                 \
    _Pragma("unroll") for (int g = 0; g < 8; ++g) P[g] = xw[tile(IT) + g * 64]; \
  }
  auto compute = [&](int buf, float4 (&x)[8]) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      float4 w0, w1;
      if (MODE == 5 || MODE == 6) {
        const float4* wp = buf ? Wb : Wa;
        w0 = wp[(2 * g) * 64 + lane];
        w1 = wp[(2 * g + 1) * 64 + lane];
      } else if (MODE >= 2) {
        w0 = Wl[buf * 1024 + (2 * g) * 64 + lane];
        w1 = Wl[buf * 1024 + (2 * g + 1) * 64 + lane];
      } else {
        w0 = x[(g + 1) & 7];
        w1 = x[(g + 3) & 7];
      }
      STEP(w0, w1, x[g])
    }
    if (MODE == 9 || MODE == 10) {
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      }
    }
  };
  auto loadw = [&](int it, int buf) {
    if ((MODE >= 7)) {
      const int off = (int)(((unsigned)((blockIdx.x + 7 * it) % 175) * 1024u + threadIdx.x) * 16u);
      float4* d = Wl + buf * 1024 + (threadIdx.x & ~63);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void*)(d + 256 * j), 16, off,
                                                 j * 4096, 0, 0);
      return;
    }
    const float4* ws = W + (size_t)((blockIdx.x + 7 * it) % 175) * 1024 + threadIdx.x;
    float4* d = ((MODE == 5 || MODE == 6) ? (buf ? Wb : Wa) : Wl + buf * 1024) + (threadIdx.x & ~63);
    GLDS(ws, d) GLDS(ws + 256, d + 256) GLDS(ws + 512, d + 512) GLDS(ws + 768, d + 768)
  };
#define SGB(MASK, N) __builtin_amdgcn_sched_group_barrier(MASK, N, 0);
  // 12 x (1 VMEM read, 5 MFMA), then the remaining 4 MFMAs
#define SPREAD                                                                           \
  if (MODE == 6 || MODE == 8) {                                                          \
    SGB(0x020, 1) SGB(0x008, 5) SGB(0x020, 1) SGB(0x008, 5) SGB(0x020, 1) SGB(0x008, 5)  \
    SGB(0x020, 1) SGB(0x008, 5) SGB(0x020, 1) SGB(0x008, 5) SGB(0x020, 1) SGB(0x008, 5)  \
    SGB(0x020, 1) SGB(0x008, 5) SGB(0x020, 1) SGB(0x008, 5) SGB(0x020, 1) SGB(0x008, 5)  \
    SGB(0x020, 1) SGB(0x008, 5) SGB(0x020, 1) SGB(0x008, 5) SGB(0x020, 1) SGB(0x008, 5)  \
    SGB(0x008, 4)                                                                        \
  }
#define STEP2(W0, W1, XV)                \
  acc2 = MFMA32((W0).x, (XV).x, acc2);   \
  acc3 = MFMA32((W1).x, (XV).x, acc3);   \
  acc2 = MFMA32((W0).y, (XV).y, acc2);   \
  acc3 = MFMA32((W1).y, (XV).y, acc3);   \
  acc2 = MFMA32((W0).z, (XV).z, acc2);   \
  acc3 = MFMA32((W1).z, (XV).z, acc3);   \
  acc2 = MFMA32((W0).w, (XV).w, acc2);   \
  acc3 = MFMA32((W1).w, (XV).w, acc3);
  auto compute2 = [&](int buf, float4 (&x)[8]) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const float4 w0 = Wl[buf * 1024 + (2 * g) * 64 + lane];
      const float4 w1 = Wl[buf * 1024 + (2 * g + 1) * 64 + lane];
      STEP2(w0, w1, x[g])
    }
    // two fragment reads ahead of each group of eight MFMAs (keeps the reads from
    // being hoisted into one block of 64 registers)
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
  };
  if (MODE >= 11 && MODE <= 13) {
    const float* L = (const float*)Wl;  // As[2][64 * 36], Ds[64 * 36] floats: 27 KB of the 32 KB
    const int lr = lane & 31, h = lane >> 5, bi = w >> 1, hp = w & 1;
    const float* Ap = L + bi * 2304 + (32 * hp + lr) * 36 + 4 * h;
    const float* D0 = L + 4608 + lr * 36 + 4 * h;
    const float* D1 = L + 4608 + (32 + lr) * 36 + 4 * h;
    for (int it = 0; it < iters; ++it) {
      if (MODE <= 12) __syncthreads();
      if (MODE == 11) __syncthreads();
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 av = *(const float4*)(Ap + 8 * g);
        const float4 d0 = *(const float4*)(D0 + 8 * g);
        const float4 d1 = *(const float4*)(D1 + 8 * g);
        acc0 = MFMA32(av.x, d0.x, acc0); acc1 = MFMA32(av.x, d1.x, acc1);
        acc0 = MFMA32(av.y, d0.y, acc0); acc1 = MFMA32(av.y, d1.y, acc1);
        acc0 = MFMA32(av.z, d0.z, acc0); acc1 = MFMA32(av.z, d1.z, acc1);
        acc0 = MFMA32(av.w, d0.w, acc0); acc1 = MFMA32(av.w, d1.w, acc1);
      }
    }
  } else
  if (MODE == 9 || MODE == 10) {
    // iterations come in fours: (xa, slab 0) (xa, slab 1) (xb, slab 0) (xb, slab 1)
    for (int it = 0; it < iters; it += 4) {
      loadw(it + 1, 1);
      LOADXM(xb, it + 2)
      compute(0, xa);
      __syncthreads();
      loadw(it + 2, 0);
      if (MODE == 10) { LOADXM(xa, it + 3) }
      compute2(1, MODE == 10 ? xb : xa);
      __syncthreads();
      loadw(it + 3, 1);
      LOADXM(xa, it + 4)
      compute(0, MODE == 10 ? xa : xb);
      __syncthreads();
      loadw(it + 4, 0);
      if (MODE == 10) { LOADXM(xb, it + 5) }
      compute2(1, xb);
      __syncthreads();
    }
  } else
  for (int it = 0; it < iters; it += 2) {
    if (MODE >= 4) loadw(it + 1, 1);
    LOADXM(xb, it + 1)
    compute(0, xa);
    SPREAD
    if (MODE == 5 || MODE == 6) __builtin_amdgcn_s_waitcnt(0x0F70);
    if (MODE >= 1) __syncthreads();
    if (MODE >= 4) loadw(it + 2, 0);
    LOADXM(xa, it + 2)
    compute(1, xb);
    SPREAD
    if (MODE == 5 || MODE == 6) __builtin_amdgcn_s_waitcnt(0x0F70);
    if (MODE >= 1) __syncthreads();
  }
  float s = 0.f;
  for (int k = 0; k < 16; ++k) s += acc0[k] + acc1[k] + acc2[k] + acc3[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE, int WPE = 4>
static void run(int iters, const float4* X, const float4* W, int n_tiles, float* out, int grid) {
  grid = grid / 4 * WPE;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((loop_kernel<MODE, WPE>), dim3(grid), dim3(256), 2 * 1024 * sizeof(float4), 0, iters, X, W, n_tiles, out);
    (void)hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) { std::printf("mode %d failed\n", MODE); return; }
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  const double flop = (double)grid * 4 * iters * (MODE >= 11 && MODE <= 13 ? 32 : 64) * 4096.0;
  std::printf("mode %d (%d workgroups per CU): %.2f ms, %.1f TFLOP/s (%.1f%% of 157.3)\n", MODE, WPE, best, flop / (best * 1e-3) / 1e12,
              100.0 * flop / (best * 1e-3) / 1e12 / 157.3);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int n_tiles = argc > 2 ? std::atoi(argv[2]) : 34816;  // 285 MB of activations (2048 row tiles x 17 slabs)
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  const int grid = p.multiProcessorCount * 4;
  float4 *X, *W;
  float* out;
  if (hipMalloc(&X, (size_t)n_tiles * 512 * 16) != hipSuccess) return 1;
  if (hipMalloc(&W, (size_t)175 * 1024 * 16) != hipSuccess) return 1;
  if (hipMalloc(&out, (size_t)grid * 256 * 4) != hipSuccess) return 1;
  (void)hipMemset(X, 0, (size_t)n_tiles * 512 * 16);
  (void)hipMemset(W, 0, (size_t)175 * 1024 * 16);
  run<0>(iters, X, W, n_tiles, out, grid);
  run<1>(iters, X, W, n_tiles, out, grid);
  run<2>(iters, X, W, n_tiles, out, grid);
  run<3>(iters, X, W, n_tiles, out, grid);
  run<4>(iters, X, W, n_tiles, out, grid);
  run<5>(iters, X, W, n_tiles, out, grid);
  run<6>(iters, X, W, n_tiles, out, grid);
  run<7>(iters, X, W, n_tiles, out, grid);
  run<8>(iters, X, W, n_tiles, out, grid);
  run<7, 3>(iters, X, W, n_tiles, out, grid);
  run<8, 3>(iters, X, W, n_tiles, out, grid);
  run<11>(iters, X, W, n_tiles, out, grid);
  run<12>(iters, X, W, n_tiles, out, grid);
  run<13>(iters, X, W, n_tiles, out, grid);
  run<11, 3>(iters, X, W, n_tiles, out, grid);
  run<11, 5>(iters, X, W, n_tiles, out, grid);
  run<9, 3>(iters, X, W, n_tiles, out, grid);
  run<10, 3>(iters, X, W, n_tiles, out, grid);
  run<9, 2>(iters, X, W, n_tiles, out, grid);
  run<10, 2>(iters, X, W, n_tiles, out, grid);
  run<7, 2>(iters, X, W, n_tiles, out, grid);
  run<8, 2>(iters, X, W, n_tiles, out, grid);
  return 0;
}
