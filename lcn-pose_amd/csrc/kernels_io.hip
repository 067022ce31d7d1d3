// Output assembly and loss of the LCN (gfx950).
//
// The thin layers themselves (lift x.W1e, output h.W4e and their gradients)
// run on the block-sparse MFMA kernels with the narrow side padded to one
// 64-wide slab (see lcn_api.cpp); what remains here is the elementwise tail of
// the output layer (models_att.py:768-773) and the MSE loss (:356) with its
// gradient d out = 2 (out - lab) / (B * 51).
#include <algorithm>

#include "lcn_internal.h"

namespace lcn {

// One wave per row (lane = output column, 51 of 64 active), grid-stride rows;
// y, x and dy are 1-slab row-tiled buffers (lcn_internal.h), out / lab row-major.
__global__ __launch_bounds__(256) void out_assemble_kernel(OutAsmArgs a) {
  __shared__ double red[4];
  __shared__ double dred[4][64];
  const int t = threadIdx.x, c = t & 63, w = t >> 6;
  const int j = c / 3, k = c - 3 * j;
  // d out = 2 (out - lab) / (rows * 51), rows over all ranks
  const float dscale = (float)(2.0 / ((a.ri ? a.ri->rows_global : a.rows) * 51.0));
  double lsum = 0.0, dsum = 0.0;  // dsum: this lane's column of dy over its rows (db4 = sum_b dy)
  for (int row = blockIdx.x * 4 + w; row < a.B; row += gridDim.x * 4) {
    if (c < 51) {
      const float y = a.y[tix(row, c, 1)] + a.b4[c];
      const float o = k < 2 ? a.x[tix(row, a.in_f * j + k, 1)] + y : y;
      a.out[(size_t)row * 51 + c] = o;
      if (a.lab) {
        const float d = o - a.lab[(size_t)row * 51 + c];
        lsum += (double)d * (double)d;
        if (a.dy) {
          const float g = dscale * d;
          a.dy[tix(row, c, 1)] = g;
          dsum += (double)g;
        }
      }
    } else if (a.dy) {
      a.dy[tix(row, c, 1)] = 0.f;  // padded columns of the output layer's dX operand
    }
  }
  if (!a.loss_part) return;
  for (int o = 32; o > 0; o >>= 1) lsum += __shfl_xor(lsum, o);
  if (c == 0) red[w] = lsum;
  dred[w][c] = dsum;
  __syncthreads();
  if (t == 0) a.loss_part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  if (a.db_part && w == 0) a.db_part[blockIdx.x * 64 + c] = (dred[0][c] + dred[1][c]) + (dred[2][c] + dred[3][c]);
}

void launch_out_assemble(const OutAsmArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(out_assemble_kernel, dim3(grid), dim3(256), 0, s, a);
}

// row-major [B][cols] -> 1-slab row tiles, zero padded; one thread per float4
__global__ __launch_bounds__(256) void tile_in_kernel(const float* __restrict__ src, int cols,
                                                      int B, float4* __restrict__ dst, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(i & 511), l = c4 & 63;
    const int64_t row = (i >> 9) * kRT + (l & 31);
    const int c = 8 * (c4 >> 6) + 4 * (l >> 5);
    float v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) v[s] = (row < B && c + s < cols) ? src[row * cols + c + s] : 0.f;
    dst[i] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

void launch_tile_in(const float* src, int cols, int B, float* dst, hipStream_t s) {
  const int64_t n4 = tiled_floats(B, 1) / 4;
  const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 4096);
  hipLaunchKernelGGL(tile_in_kernel, dim3(grid), dim3(256), 0, s, src, cols, B, (float4*)dst, n4);
}

// workgroup 0: the loss; workgroup 1 + c: column c of dy -> db_out[c]
__global__ __launch_bounds__(256) void loss_finalize_kernel(const double* part, int n, double* out,
                                                            const double* db_part, float* db_out) {
  __shared__ double red[256];
  const int b = blockIdx.x;
  double s = 0.0;
  if (b == 0) {
    for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  } else {
    for (int i = threadIdx.x; i < n; i += 256) s += db_part[(size_t)i * 64 + (b - 1)];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (b == 0) out[0] = red[0];
    else db_out[b - 1] = (float)red[0];
  }
}

void launch_loss_finalize(const double* part, int n, double* out, const double* db_part, float* db_out,
                          hipStream_t s) {
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(db_part ? 52 : 1), dim3(256), 0, s, part, n, out, db_part,
                     db_out);
}

}  // namespace lcn
