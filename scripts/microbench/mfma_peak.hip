// What the fp32 MFMA pipe sustains on this part: every SIMD runs `waves` waves
// that issue nothing but v_mfma_f32_32x32x2_f32 on two alternating
// accumulators (the block-sparse GEMMs' inner pattern), for about a second.
// Reports TFLOP/s against the 157.3 TFLOP/s data-sheet peak and the shader
// clock over the run (s_memtime / s_memrealtime), i.e. how much of the peak is
// clock (power management under sustained matrix load) rather than issue.
//   hipcc --offload-arch=gfx950 -O3 -o mfma_peak mfma_peak.hip && ./mfma_peak [waves_per_simd] [iters]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma_loop(int iters, float* out, uint64_t* stamps) {
  const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  f32x16 a0, a1;
  for (int k = 0; k < 16; ++k) { a0[k] = 0.f; a1[k] = 0.f; }
  // 16 + 16 operand registers of hashed values per lane, cycled through, so the
  // operand buses toggle as they do on real data
  float xr[16], wr[16];
  unsigned hsh = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
  for (int k = 0; k < 16; ++k) {
    hsh = hsh * 1664525u + 1013904223u;
    xr[k] = (float)(int)(hsh >> 8) * (1.0f / 8388608.0f) - 1.0f;
    hsh = hsh * 1664525u + 1013904223u;
    wr[k] = ((float)(int)(hsh >> 8) * (1.0f / 8388608.0f) - 1.0f) * 1e-3f;
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[j & 15], xr[j & 15], a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[(j + 5) & 15], xr[(j + 3) & 15], a1, 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int k = 0; k < 16; ++k) s += a0[k] + a1[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
    stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

int main(int argc, char** argv) {
  const int waves = argc > 1 ? std::atoi(argv[1]) : 4;  // per SIMD; a 256-thread workgroup = 1 wave per SIMD
  const int iters = argc > 2 ? std::atoi(argv[2]) : 40000;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  const int grid = p.multiProcessorCount * waves;
  float* out;
  uint64_t* st;
  hipMalloc(&out, (size_t)grid * 256 * 4);
  hipMalloc(&st, (size_t)grid * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(mfma_loop, dim3(grid), dim3(256), 0, 0, iters, out, st);
    hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) return 2;
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> h((size_t)grid * 2);
    hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    double ghz = 0;
    for (int i = 0; i < grid; ++i) ghz += (double)h[2 * i] / (double)h[2 * i + 1] * 0.1;
    const double flop = (double)grid * 4 * iters * 64 * 4096.0;
    std::printf("CUs %d, %d waves/SIMD: %.1f ms, %.1f TFLOP/s (%.1f%% of 157.3), shader clock %.3f GHz\n",
                p.multiProcessorCount, waves, ms, flop / (ms * 1e-3) / 1e12,
                100.0 * flop / (ms * 1e-3) / 1e12 / 157.3, ghz / grid);
  }
  return 0;
}
