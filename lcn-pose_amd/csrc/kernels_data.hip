// Device-resident datasets: permutation gather, test-time augmentation and
// its undo (gfx950).
//
// The reference feeds every step from the host: fit() draws batch indices
// from a deque of np.random.permutation()s and fancy-indexes the float64
// train arrays (models_att.py:193-200); predict() slices fixed batches,
// zero-pads the last one (:88-97) and feeds them; inference.py concatenates
// flipped / rotated / translated copies of the test set before predict and
// averages the undone copies after it (inference.py:70-110, data.py:10-54,
// 205-322).  Here the arrays stay in HBM in the dtype the caller gave
// (float64 in the reference pipeline) and a batch is built on the device:
//
//   * the "virtual" row v of a batch addresses the concatenation of n_copies
//     augmented copies of the dataset (copy c = v / N, row r = v % N), exactly
//     the array inference.py would have concatenated; v outside [0, c*N) is a
//     zero row (predict's zero padding, which enters the BN statistics);
//   * the augmentation of copy c is applied in float64 with the reference's
//     operation order, then rounded to float32 -- the same value a float32
//     placeholder receives from the reference's float64 array (feed_dict
//     casting = round to nearest even);
//   * the result lands directly in the lift GEMM's 1-slab row-tiled operand.
//
// All of these are HBM/latency-bound byte movers: one thread per output
// float4, coalesced writes, rows read through L2.
#include <algorithm>

#include "lcn_internal.h"

namespace lcn {

// flip_data's joint permutation (data.py:18-22): LEFT = 4,5,6,11,12,13 and
// RIGHT = 1,2,3,14,15,16 swap places; every other joint maps to itself
__device__ __forceinline__ int flip_src(int j) {
  switch (j) {
    case 1: return 4;  case 2: return 5;  case 3: return 6;
    case 4: return 1;  case 5: return 2;  case 6: return 3;
    case 11: return 14; case 12: return 15; case 13: return 16;
    case 14: return 11; case 15: return 12; case 16: return 13;
    default: return j;
  }
}

__device__ __forceinline__ double ds_at(const void* ds, int dtype, int64_t i) {
  return dtype == kF64 ? ((const double*)ds)[i] : (double)((const float*)ds)[i];
}

// value of feature col (= k*j + c) of augmented row r under op (float64)
__device__ __forceinline__ double aug_value(const void* ds, int dtype, int64_t r, int k, int col,
                                            int op, double p0, double p1) {
  const int64_t base = r * (int64_t)(kJ * k);
  const int j = col / k, c = col - j * k;
  if (op == kAugFlip) {  // data.py:21-22: x of every joint negated, then L/R swapped
    const double v = ds_at(ds, dtype, base + flip_src(j) * k + c);
    return c == 0 ? -v : v;
  }
  if (op == kAugTranslate) {  // data.py:46-52: x, y (and the third channel) + t
    return ds_at(ds, dtype, base + col) + p0;
  }
  if (op == kAugRotate) {
    // data.py:298-318: rotation about the z axis around joint 0,
    // p' = (p - pivot) @ Rz^T (the 2x2 block for two channels) + pivot, with
    // p0 = cos(theta), p1 = sin(theta) computed by the caller exactly as numpy
    // does.  Rz^T = [[c, s, 0], [-s, c, 0], [0, 0, 1]]; the dot products are
    // accumulated k-ascending with fma as BLAS dgemm does.
    const double px = ds_at(ds, dtype, base + 0), py = ds_at(ds, dtype, base + 1);
    const double dx = ds_at(ds, dtype, base + j * k + 0) - px;
    const double dy = ds_at(ds, dtype, base + j * k + 1) - py;
    if (c == 0) return fma(dy, -p1, dx * p0) + px;
    if (c == 1) return fma(dy, p0, dx * p1) + py;
    const double pz = ds_at(ds, dtype, base + 2);
    return (ds_at(ds, dtype, base + j * k + 2) - pz) + pz;
  }
  return ds_at(ds, dtype, base + col);
}

struct GatherArgs {
  const void* ds; int dtype; int64_t rows; int k;   // dataset [rows][17*k]
  const int* idx; int64_t base;                      // v = idx ? idx[b] : base + b
  Augment aug;                                       // copies of the virtual array
  int B;
  float4* dst;                                       // 1-slab row tiles (tiled_floats(B, 1))
  int64_t n4;
};

__global__ __launch_bounds__(256) void gather_x_kernel(GatherArgs a) {
  const int cols = kJ * a.k;
  const int64_t total = a.rows * a.aug.n_copies;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n4; i += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(i & 511), l = c4 & 63;
    const int64_t b = (i >> 9) * kRT + (l & 31);
    const int col = 8 * (c4 >> 6) + 4 * (l >> 5);
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (b < a.B && col < cols) {
      const int64_t vr = a.idx ? (int64_t)a.idx[b] : a.base + b;
      if (vr >= 0 && vr < total) {
        const int cp = (int)(vr / a.rows);
        const int64_t r = vr - (int64_t)cp * a.rows;
        const int op = a.aug.op[cp];
        const double p0 = a.aug.p0[cp], p1 = a.aug.p1[cp];
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (col + s < cols) v[s] = (float)aug_value(a.ds, a.dtype, r, a.k, col + s, op, p0, p1);
      }
    }
    a.dst[i] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

void launch_gather_x(const void* ds, int dtype, int64_t rows, int k, const int* idx, int64_t base,
                     const Augment& aug, int B, float* dst, hipStream_t s) {
  GatherArgs a{ds, dtype, rows, k, idx, base, aug, B, (float4*)dst, tiled_floats(B, 1) / 4};
  const int grid = (int)std::min<int64_t>((a.n4 + 255) / 256, 4096);
  hipLaunchKernelGGL(gather_x_kernel, dim3(grid), dim3(256), 0, s, a);
}

// row-major gather of `cols` columns: dst[b][c] = float(ds[v][c]), 0 outside
__global__ __launch_bounds__(256) void gather_rows_kernel(const void* __restrict__ ds, int dtype,
                                                          int64_t rows, int cols,
                                                          const int* __restrict__ idx, int64_t base,
                                                          int B, float* __restrict__ dst) {
  const int64_t n = (int64_t)B * cols;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / cols;
    const int c = (int)(i - b * cols);
    const int64_t v = idx ? (int64_t)idx[b] : base + b;
    dst[i] = (v >= 0 && v < rows) ? (float)ds_at(ds, dtype, v * cols + c) : 0.f;
  }
}

void launch_gather_rows(const void* ds, int dtype, int64_t rows, int cols, const int* idx,
                        int64_t base, int B, float* dst, hipStream_t s) {
  const int64_t n = (int64_t)B * cols;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid), dim3(256), 0, s, ds, dtype, rows, cols, idx,
                     base, B, dst);
}

// predictions of one batch (float32 [B][51]) -> rows [begin, begin + n) of the
// float64 prediction array (predict's `predictions[begin:end] = batch_pred`)
__global__ __launch_bounds__(256) void store_pred_kernel(const float* __restrict__ out, int64_t n,
                                                         double* __restrict__ pred) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n * 51; i += (int64_t)gridDim.x * 256)
    pred[i] = (double)out[i];
}

void launch_store_pred(const float* out, int64_t n, double* pred, hipStream_t s) {
  const int grid = (int)std::min<int64_t>((n * 51 + 255) / 256, 4096);
  hipLaunchKernelGGL(store_pred_kernel, dim3(grid), dim3(256), 0, s, out, n, pred);
}

// data.undo (data.py:269-287): copy c of the [(n_copies) N][17][3] predictions
// is un-augmented (unflip :236-249, rotate_data :289-322 with the undo angle,
// untranslation :205-218 -- which subtracts t from all three coordinates),
// then the copies are averaged as np.mean(axis=0) does: ((p0 + p1) + p2) / n.
// One thread per (row, joint); float64 throughout.
__global__ __launch_bounds__(256) void tta_undo_kernel(const double* __restrict__ pred, int64_t N,
                                                       Augment undo, double* __restrict__ out) {
  const int64_t n = N * kJ;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / kJ;
    const int j = (int)(i - r * kJ);
    double acc[3];
    for (int cp = 0; cp < undo.n_copies; ++cp) {
      const double* P = pred + ((int64_t)cp * N + r) * 51;
      double q[3];
      const int op = undo.op[cp];
      if (op == kAugFlip) {
        const int js = flip_src(j);
        q[0] = -P[3 * js]; q[1] = P[3 * js + 1]; q[2] = P[3 * js + 2];
      } else if (op == kAugRotate) {
        const double c = undo.p0[cp], s = undo.p1[cp];
        const double dx = P[3 * j] - P[0], dy = P[3 * j + 1] - P[1], dz = P[3 * j + 2] - P[2];
        // (p - pivot) @ Rz^T with Rz^T rows (c, s, 0), (-s, c, 0), (0, 0, 1)
        q[0] = fma(dz, 0.0, fma(dy, -s, dx * c)) + P[0];
        q[1] = fma(dz, 0.0, fma(dy, c, dx * s)) + P[1];
        q[2] = fma(dz, 1.0, fma(dy, 0.0, dx * 0.0)) + P[2];
      } else if (op == kAugTranslate) {
        q[0] = P[3 * j] - undo.p0[cp]; q[1] = P[3 * j + 1] - undo.p0[cp]; q[2] = P[3 * j + 2] - undo.p0[cp];
      } else {
        q[0] = P[3 * j]; q[1] = P[3 * j + 1]; q[2] = P[3 * j + 2];
      }
      if (cp == 0) { acc[0] = q[0]; acc[1] = q[1]; acc[2] = q[2]; }
      else { acc[0] += q[0]; acc[1] += q[1]; acc[2] += q[2]; }
    }
    const double nc = (double)undo.n_copies;
    out[r * 51 + 3 * j + 0] = acc[0] / nc;
    out[r * 51 + 3 * j + 1] = acc[1] / nc;
    out[r * 51 + 3 * j + 2] = acc[2] / nc;
  }
}

void launch_tta_undo(const double* pred, int64_t N, const Augment& undo, double* out, hipStream_t s) {
  const int grid = (int)std::min<int64_t>((N * kJ + 255) / 256, 4096);
  hipLaunchKernelGGL(tta_undo_kernel, dim3(grid), dim3(256), 0, s, pred, N, undo, out);
}

// per-batch predict loss (float32, as the reference's fetched batch_loss):
// losses[i] = (float)(loss_sum / (rows * 51)), rows over all ranks
__global__ void batch_loss_kernel(const double* loss_sum, double rows, const RowInfo* ri,
                                  float* losses, int i) {
  if (threadIdx.x == 0) losses[i] = (float)(loss_sum[0] / ((ri ? ri->rows_global : rows) * 51.0));
}

void launch_batch_loss(const double* loss_sum, double rows, const RowInfo* ri, float* losses, int i,
                       hipStream_t s) {
  hipLaunchKernelGGL(batch_loss_kernel, dim3(1), dim3(64), 0, s, loss_sum, rows, ri, losses, i);
}

}  // namespace lcn
