// Prototype: block-sparse fp32 MFMA GEMM on a fragment-tiled activation layout
// (no LDS, no barriers).  Stand-alone timing at the cfg3 shape.
//   activations X[rt32][slab][g][lane][4]: 32 rows x 64 features per 8 KB tile,
//     chunk g (1 KB) holds, for lane l, row (l&31), features 8g + 4(l>>5) + 0..3
//   blocks W[blk][g][half][lane][4] = We[n = 32 half + (l&31)][k = 8g + 4(l>>5) + s]
// MFMA roles swapped (D[n][b] = sum_k We[n][k] X[b][k]): the accumulator of a
// lane is then 4 consecutive features of one row = the tiled chunk layout.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

#define STEP(W0, W1, X)                 \
  acc0 = MFMA32((W0).x, (X).x, acc0);   \
  acc1 = MFMA32((W1).x, (X).x, acc1);   \
  acc0 = MFMA32((W0).y, (X).y, acc0);   \
  acc1 = MFMA32((W1).y, (X).y, acc1);   \
  acc0 = MFMA32((W0).z, (X).z, acc0);   \
  acc1 = MFMA32((W1).z, (X).z, acc1);   \
  acc0 = MFMA32((W0).w, (X).w, acc0);   \
  acc1 = MFMA32((W1).w, (X).w, acc1);

#define DECL(P) float4 P##x0, P##x1, P##x2, P##x3, P##x4, P##x5, P##x6, P##x7, \
  P##w0, P##w1, P##w2, P##w3, P##w4, P##w5, P##w6, P##w7, P##w8, P##w9, P##w10, P##w11, \
  P##w12, P##w13, P##w14, P##w15;
#define LOAD(P, E)                                                    \
  {                                                                   \
    const int2 ib_ = idx[(E)];                                        \
    const float4* xs_ = xw + (size_t)ib_.x * 512;                     \
    const float4* ws_ = W4 + (size_t)ib_.y * 1024 + lane;             \
    P##x0 = xs_[0]; P##x1 = xs_[64]; P##x2 = xs_[128]; P##x3 = xs_[192]; \
    P##x4 = xs_[256]; P##x5 = xs_[320]; P##x6 = xs_[384]; P##x7 = xs_[448]; \
    P##w0 = ws_[0]; P##w1 = ws_[64]; P##w2 = ws_[128]; P##w3 = ws_[192]; \
    P##w4 = ws_[256]; P##w5 = ws_[320]; P##w6 = ws_[384]; P##w7 = ws_[448]; \
    P##w8 = ws_[512]; P##w9 = ws_[576]; P##w10 = ws_[640]; P##w11 = ws_[704]; \
    P##w12 = ws_[768]; P##w13 = ws_[832]; P##w14 = ws_[896]; P##w15 = ws_[960]; \
  }
#define COMPUTE(P)                         \
  STEP(P##w0, P##w1, P##x0)                \
  STEP(P##w2, P##w3, P##x1)                \
  STEP(P##w4, P##w5, P##x2)                \
  STEP(P##w6, P##w7, P##x3)                \
  STEP(P##w8, P##w9, P##x4)                \
  STEP(P##w10, P##w11, P##x5)              \
  STEP(P##w12, P##w13, P##x6)              \
  STEP(P##w14, P##w15, P##x7)

// one wave = 32 rows x one 64-wide output slab; 4 waves of a workgroup take 4
// consecutive row tiles of the same output slab (W shared through L1)
__global__ __launch_bounds__(256, 2) void tiled_fwd(const float4* __restrict__ X, int S_in,
                                                    const float4* __restrict__ W4,
                                                    const int* __restrict__ ptr,
                                                    const int2* __restrict__ idx,
                                                    const float* __restrict__ bias,
                                                    float4* __restrict__ Y, int S_out,
                                                    int n_out, int n_rt32) {
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int rtg = wg / n_out, so = wg - rtg * n_out;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rt = rtg * 4 + w;
  if (rt >= n_rt32) return;
  const int beg = ptr[so], end = ptr[so + 1];
  const float4* xw = X + (size_t)rt * S_in * 512 + lane;
  f32x16 acc0, acc1;
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; }
  DECL(a)
  DECL(b)
  LOAD(a, beg)
  for (int e = beg; e < end; e += 2) {
    if (e + 1 < end) LOAD(b, e + 1)
    COMPUTE(a)
    if (e + 1 < end) {
      if (e + 2 < end) LOAD(a, e + 2)
      COMPUTE(b)
    }
  }
  const int h = lane >> 5;
  const float* bs = bias + so * 64 + 4 * h;
  float4* yo = Y + ((size_t)rt * S_out + so) * 512 + lane;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 b0 = *(const float4*)(bs + 8 * q), b1 = *(const float4*)(bs + 32 + 8 * q);
    yo[q * 64] = make_float4(acc0[4 * q] + b0.x, acc0[4 * q + 1] + b0.y, acc0[4 * q + 2] + b0.z,
                             acc0[4 * q + 3] + b0.w);
    yo[(4 + q) * 64] = make_float4(acc1[4 * q] + b1.x, acc1[4 * q + 1] + b1.y,
                                   acc1[4 * q + 2] + b1.z, acc1[4 * q + 3] + b1.w);
  }
}

// V1: X fragments direct to registers (tiled layout), W block through LDS
// (double buffered, one barrier per input slab, shared by the 4 waves)
#define DECLX(P) float4 P##0, P##1, P##2, P##3, P##4, P##5, P##6, P##7;
#define LOADX(P, E)                                                        \
  {                                                                        \
    const float4* xs_ = xw + (size_t)idx[(E)].x * 512;                     \
    P##0 = xs_[0]; P##1 = xs_[64]; P##2 = xs_[128]; P##3 = xs_[192];       \
    P##4 = xs_[256]; P##5 = xs_[320]; P##6 = xs_[384]; P##7 = xs_[448];    \
  }
#define LOADW(E)                                                           \
  {                                                                        \
    const float4* ws_ = W4 + (size_t)idx[(E)].y * 1024 + threadIdx.x;      \
    st0 = ws_[0]; st1 = ws_[256]; st2 = ws_[512]; st3 = ws_[768];          \
  }
#define STOREW(BUF)                                                        \
  {                                                                        \
    float4* d_ = Wl + (BUF) * 1024 + threadIdx.x;                          \
    d_[0] = st0; d_[256] = st1; d_[512] = st2; d_[768] = st3;              \
  }
#define GSTEP(BUF, G, XV)                                                  \
  {                                                                        \
    const float4 w0_ = Wl[(BUF) * 1024 + (2 * (G)) * 64 + lane];           \
    const float4 w1_ = Wl[(BUF) * 1024 + (2 * (G) + 1) * 64 + lane];       \
    STEP(w0_, w1_, XV)                                                     \
  }
#define COMPX(BUF, P)                                                      \
  GSTEP(BUF, 0, P##0) GSTEP(BUF, 1, P##1) GSTEP(BUF, 2, P##2) GSTEP(BUF, 3, P##3) \
  GSTEP(BUF, 4, P##4) GSTEP(BUF, 5, P##5) GSTEP(BUF, 6, P##6) GSTEP(BUF, 7, P##7)

__global__ __launch_bounds__(256) void tiled_fwd_ldsw(const float4* __restrict__ X, int S_in,
                                                      const float4* __restrict__ W4,
                                                      const int* __restrict__ ptr,
                                                      const int2* __restrict__ idx,
                                                      const float* __restrict__ bias,
                                                      float4* __restrict__ Y, int S_out,
                                                      int n_out, int n_rt32) {
  __shared__ float4 Wl[2 * 1024];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int rtg = wg / n_out, so = wg - rtg * n_out;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rt = min(rtg * 4 + w, n_rt32 - 1);  // clamped: every wave takes part in the barriers
  const int beg = ptr[so], end = ptr[so + 1];
  const float4* xw = X + (size_t)rt * S_in * 512 + lane;
  f32x16 acc0, acc1;
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; }
  float4 st0, st1, st2, st3;
  DECLX(xa)
  DECLX(xb)
  LOADW(beg)
  LOADX(xa, beg)
  STOREW(0)
  __syncthreads();
  for (int e = beg; e < end; e += 2) {
    if (e + 1 < end) { LOADW(e + 1) LOADX(xb, e + 1) }
    COMPX(0, xa)
    if (e + 1 < end) STOREW(1)
    __syncthreads();
    if (e + 1 < end) {
      if (e + 2 < end) { LOADW(e + 2) LOADX(xa, e + 2) }
      COMPX(1, xb)
      if (e + 2 < end) STOREW(0)
      __syncthreads();
    }
  }
  if (rtg * 4 + w >= n_rt32) return;
  const int h = lane >> 5;
  const float* bs = bias + so * 64 + 4 * h;
  float4* yo = Y + ((size_t)rt * S_out + so) * 512 + lane;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 b0 = *(const float4*)(bs + 8 * q), b1 = *(const float4*)(bs + 32 + 8 * q);
    yo[q * 64] = make_float4(acc0[4 * q] + b0.x, acc0[4 * q + 1] + b0.y, acc0[4 * q + 2] + b0.z,
                             acc0[4 * q + 3] + b0.w);
    yo[(4 + q) * 64] = make_float4(acc1[4 * q] + b1.x, acc1[4 * q + 1] + b1.y,
                                   acc1[4 * q + 2] + b1.z, acc1[4 * q + 3] + b1.w);
  }
}

// V2: as V1, each wave 64 rows (two 32-row tiles, 4 accumulators): every W
// fragment read from LDS feeds 4 MFMAs instead of 2
#define STEP2(W0, W1, X, Y)               \
  acc0 = MFMA32((W0).x, (X).x, acc0);     \
  acc1 = MFMA32((W1).x, (X).x, acc1);     \
  acc2 = MFMA32((W0).x, (Y).x, acc2);     \
  acc3 = MFMA32((W1).x, (Y).x, acc3);     \
  acc0 = MFMA32((W0).y, (X).y, acc0);     \
  acc1 = MFMA32((W1).y, (X).y, acc1);     \
  acc2 = MFMA32((W0).y, (Y).y, acc2);     \
  acc3 = MFMA32((W1).y, (Y).y, acc3);     \
  acc0 = MFMA32((W0).z, (X).z, acc0);     \
  acc1 = MFMA32((W1).z, (X).z, acc1);     \
  acc2 = MFMA32((W0).z, (Y).z, acc2);     \
  acc3 = MFMA32((W1).z, (Y).z, acc3);     \
  acc0 = MFMA32((W0).w, (X).w, acc0);     \
  acc1 = MFMA32((W1).w, (X).w, acc1);     \
  acc2 = MFMA32((W0).w, (Y).w, acc2);     \
  acc3 = MFMA32((W1).w, (Y).w, acc3);
#define GSTEP2(BUF, G, XV, YV)                                             \
  {                                                                        \
    const float4 w0_ = Wl[(BUF) * 1024 + (2 * (G)) * 64 + lane];           \
    const float4 w1_ = Wl[(BUF) * 1024 + (2 * (G) + 1) * 64 + lane];       \
    STEP2(w0_, w1_, XV, YV)                                                \
  }
#define LOADX2(P, Q, E)                                                    \
  {                                                                        \
    const float4* xs_ = xw + (size_t)idx[(E)].x * 512;                     \
    const float4* ys_ = xs_ + (size_t)S_in * 512;                          \
    P##0 = xs_[0]; P##1 = xs_[64]; P##2 = xs_[128]; P##3 = xs_[192];       \
    P##4 = xs_[256]; P##5 = xs_[320]; P##6 = xs_[384]; P##7 = xs_[448];    \
    Q##0 = ys_[0]; Q##1 = ys_[64]; Q##2 = ys_[128]; Q##3 = ys_[192];       \
    Q##4 = ys_[256]; Q##5 = ys_[320]; Q##6 = ys_[384]; Q##7 = ys_[448];    \
  }
#define COMPX2(BUF, P, Q)                                                  \
  GSTEP2(BUF, 0, P##0, Q##0) GSTEP2(BUF, 1, P##1, Q##1) GSTEP2(BUF, 2, P##2, Q##2) \
  GSTEP2(BUF, 3, P##3, Q##3) GSTEP2(BUF, 4, P##4, Q##4) GSTEP2(BUF, 5, P##5, Q##5) \
  GSTEP2(BUF, 6, P##6, Q##6) GSTEP2(BUF, 7, P##7, Q##7)

__global__ __launch_bounds__(256, 2) void tiled_fwd_ldsw2(const float4* __restrict__ X, int S_in,
                                                         const float4* __restrict__ W4,
                                                         const int* __restrict__ ptr,
                                                         const int2* __restrict__ idx,
                                                         const float* __restrict__ bias,
                                                         float4* __restrict__ Y, int S_out,
                                                         int n_out, int n_rt32) {
  __shared__ float4 Wl[2 * 1024];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int rtg = wg / n_out, so = wg - rtg * n_out;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rt = min(rtg * 8 + 2 * w, n_rt32 - 2);  // n_rt32 even here
  const int beg = ptr[so], end = ptr[so + 1];
  const float4* xw = X + (size_t)rt * S_in * 512 + lane;
  f32x16 acc0, acc1, acc2, acc3;
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; acc2[k] = 0.f; acc3[k] = 0.f; }
  float4 st0, st1, st2, st3;
  DECLX(xa)
  DECLX(ya)
  DECLX(xb)
  DECLX(yb)
  LOADW(beg)
  LOADX2(xa, ya, beg)
  STOREW(0)
  __syncthreads();
  for (int e = beg; e < end; e += 2) {
    if (e + 1 < end) { LOADW(e + 1) LOADX2(xb, yb, e + 1) }
    COMPX2(0, xa, ya)
    if (e + 1 < end) STOREW(1)
    __syncthreads();
    if (e + 1 < end) {
      if (e + 2 < end) { LOADW(e + 2) LOADX2(xa, ya, e + 2) }
      COMPX2(1, xb, yb)
      if (e + 2 < end) STOREW(0)
      __syncthreads();
    }
  }
  if (rtg * 8 + 2 * w >= n_rt32) return;
  const int h = lane >> 5;
  const float* bs = bias + so * 64 + 4 * h;
  float4* yo = Y + ((size_t)rt * S_out + so) * 512 + lane;
  float4* yo2 = yo + (size_t)S_out * 512;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 b0 = *(const float4*)(bs + 8 * q), b1 = *(const float4*)(bs + 32 + 8 * q);
    yo[q * 64] = make_float4(acc0[4 * q] + b0.x, acc0[4 * q + 1] + b0.y, acc0[4 * q + 2] + b0.z,
                             acc0[4 * q + 3] + b0.w);
    yo[(4 + q) * 64] = make_float4(acc1[4 * q] + b1.x, acc1[4 * q + 1] + b1.y,
                                   acc1[4 * q + 2] + b1.z, acc1[4 * q + 3] + b1.w);
    yo2[q * 64] = make_float4(acc2[4 * q] + b0.x, acc2[4 * q + 1] + b0.y, acc2[4 * q + 2] + b0.z,
                              acc2[4 * q + 3] + b0.w);
    yo2[(4 + q) * 64] = make_float4(acc3[4 * q] + b1.x, acc3[4 * q + 1] + b1.y,
                                    acc3[4 * q + 2] + b1.z, acc3[4 * q + 3] + b1.w);
  }
}

// V3: as V1 with one X register set refilled chunk by chunk: the load of
// chunk g of the next slab is issued right after the MFMAs that consume chunk
// g of this slab (rolling prefetch, 32 X registers instead of 64)
#define GSTEPR(BUF, G, XV, NXT)                                            \
  {                                                                        \
    const float4 w0_ = Wl[(BUF) * 1024 + (2 * (G)) * 64 + lane];           \
    const float4 w1_ = Wl[(BUF) * 1024 + (2 * (G) + 1) * 64 + lane];       \
    STEP(w0_, w1_, XV)                                                     \
    if (has_next) XV = (NXT)[(G) * 64];                                    \
  }

__global__ __launch_bounds__(256, 4) void tiled_fwd_roll(const float4* __restrict__ X, int S_in,
                                                        const float4* __restrict__ W4,
                                                        const int* __restrict__ ptr,
                                                        const int2* __restrict__ idx,
                                                        const float* __restrict__ bias,
                                                        float4* __restrict__ Y, int S_out,
                                                        int n_out, int n_rt32) {
  __shared__ float4 Wl[2 * 1024];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int rtg = wg / n_out, so = wg - rtg * n_out;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rt = min(rtg * 4 + w, n_rt32 - 1);
  const int beg = ptr[so], end = ptr[so + 1];
  const float4* xw = X + (size_t)rt * S_in * 512 + lane;
  f32x16 acc0, acc1;
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; }
  float4 st0, st1, st2, st3;
  DECLX(xa)
  LOADW(beg)
  LOADX(xa, beg)
  STOREW(0)
  __syncthreads();
  int buf = 0;
  for (int e = beg; e < end; ++e) {
    const bool has_next = e + 1 < end;
    const float4* nx = xw + (size_t)idx[has_next ? e + 1 : e].x * 512;
    if (has_next) LOADW(e + 1)
    GSTEPR(buf, 0, xa0, nx) GSTEPR(buf, 1, xa1, nx) GSTEPR(buf, 2, xa2, nx) GSTEPR(buf, 3, xa3, nx)
    GSTEPR(buf, 4, xa4, nx) GSTEPR(buf, 5, xa5, nx) GSTEPR(buf, 6, xa6, nx) GSTEPR(buf, 7, xa7, nx)
    if (has_next) STOREW(buf ^ 1)
    __syncthreads();
    buf ^= 1;
  }
  if (rtg * 4 + w >= n_rt32) return;
  const int h = lane >> 5;
  const float* bs = bias + so * 64 + 4 * h;
  float4* yo = Y + ((size_t)rt * S_out + so) * 512 + lane;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 b0 = *(const float4*)(bs + 8 * q), b1 = *(const float4*)(bs + 32 + 8 * q);
    yo[q * 64] = make_float4(acc0[4 * q] + b0.x, acc0[4 * q + 1] + b0.y, acc0[4 * q + 2] + b0.z,
                             acc0[4 * q + 3] + b0.w);
    yo[(4 + q) * 64] = make_float4(acc1[4 * q] + b1.x, acc1[4 * q + 1] + b1.y,
                                   acc1[4 * q + 2] + b1.z, acc1[4 * q + 3] + b1.w);
  }
}

static const int kNbr[17][7] = {{1, 4, 7, -1}, {0, 7, 2, -1}, {1, 3, -1}, {2, -1}, {0, 7, 5, -1},
                                {4, 6, -1}, {5, -1}, {1, 0, 4, 14, 8, 11, -1}, {7, 9, 11, 14, -1},
                                {8, 10, -1}, {9, -1}, {8, 7, 12, -1}, {11, 13, -1}, {12, -1},
                                {8, 7, 15, -1}, {14, 16, -1}, {15, -1}};

template <typename T>
T* dev(const std::vector<T>& v) {
  T* p;
  CK(hipMalloc(&p, v.size() * sizeof(T)));
  CK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? std::atoi(argv[1]) : 65536;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
  const int J = 17, F = 64, H = J * F, S = J;
  std::vector<int> A(J * J, 0);
  for (int i = 0; i < J; ++i) {
    A[i * J + i] = 1;
    for (int k = 0; kNbr[i][k] >= 0; ++k) A[i * J + kNbr[i][k]] = 1;
  }
  std::vector<int> N = A;
  for (int p = 1; p < 3; ++p) {
    std::vector<int> T(J * J, 0);
    for (int i = 0; i < J; ++i)
      for (int j = 0; j < J; ++j)
        for (int k = 0; k < J; ++k) T[i * J + j] |= N[i * J + k] && A[k * J + j];
    N = T;
  }
  std::vector<int2> blk;
  std::vector<int> bid(J * J, -1);
  for (int i = 0; i < J; ++i)
    for (int j = 0; j < J; ++j)
      if (N[j * J + i]) { bid[i * J + j] = (int)blk.size(); blk.push_back(make_int2(i, j)); }
  std::vector<int> fptr(1, 0);
  std::vector<int2> fidx;
  for (int so = 0; so < J; ++so) {
    for (int si = 0; si < J; ++si)
      if (bid[si * J + so] >= 0) fidx.push_back(make_int2(si, bid[si * J + so]));
    fptr.push_back((int)fidx.size());
  }
  const int nblk = (int)blk.size();
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  // dense row-major host data, then the tiled / packed device forms
  std::vector<float> x((size_t)B * H), wb((size_t)nblk * 4096), bias(H);
  for (auto& v : x) v = U(rng);
  for (auto& v : wb) v = U(rng) * 0.05f;
  for (auto& v : bias) v = U(rng);
  std::vector<float> xt((size_t)B * H), wt((size_t)nblk * 4096);
  for (int b = 0; b < B; ++b)
    for (int c = 0; c < H; ++c) {
      const int rt = b >> 5, sl = c >> 6, f = c & 63, g = f >> 3, hh = (f >> 2) & 1, s = f & 3;
      const int lane = (b & 31) + 32 * hh;
      xt[(((size_t)rt * S + sl) * 8 + g) * 256 + lane * 4 + s] = x[(size_t)b * H + c];
    }
  for (int k = 0; k < nblk; ++k)
    for (int n = 0; n < 64; ++n)
      for (int kk = 0; kk < 64; ++kk) {
        const int half = n >> 5, g = kk >> 3, hh = (kk >> 2) & 1, s = kk & 3;
        const int lane = (n & 31) + 32 * hh;
        wt[(size_t)k * 4096 + ((g * 2 + half) * 64 + lane) * 4 + s] = wb[(size_t)k * 4096 + n * 64 + kk];
      }
  float* dX = dev(xt);
  float* dW = dev(wt);
  float* dB = dev(bias);
  int* dptr = dev(fptr);
  int2* didx = dev(fidx);
  float* dY;
  CK(hipMalloc(&dY, (size_t)B * H * 4));
  const int n_rt32 = B / 32;
  const int grid = ((n_rt32 + 3) / 4) * J;
  int kern = 0;
  auto run = [&]() {
    if (kern == 0)
      hipLaunchKernelGGL(tiled_fwd, dim3(grid), dim3(256), 0, 0, (const float4*)dX, S,
                         (const float4*)dW, dptr, didx, dB, (float4*)dY, S, J, n_rt32);
    else if (kern == 3)
      hipLaunchKernelGGL(tiled_fwd_roll, dim3(grid), dim3(256), 0, 0, (const float4*)dX, S,
                         (const float4*)dW, dptr, didx, dB, (float4*)dY, S, J, n_rt32);
    else if (kern == 2)
      hipLaunchKernelGGL(tiled_fwd_ldsw2, dim3(((n_rt32 + 7) / 8) * J), dim3(256), 0, 0, (const float4*)dX, S,
                         (const float4*)dW, dptr, didx, dB, (float4*)dY, S, J, n_rt32);
    else
      hipLaunchKernelGGL(tiled_fwd_ldsw, dim3(grid), dim3(256), 0, 0, (const float4*)dX, S,
                         (const float4*)dW, dptr, didx, dB, (float4*)dY, S, J, n_rt32);
  };
  for (kern = 1; kern < 4; kern += 2) {
  CK(hipMemset(dY, 0, (size_t)B * H * 4));
  run();
  CK(hipDeviceSynchronize());
  // check a sample of outputs against a CPU fp64 product
  std::vector<float> yt((size_t)B * H);
  CK(hipMemcpy(yt.data(), dY, yt.size() * 4, hipMemcpyDeviceToHost));
  double maxerr = 0;
  for (int t = 0; t < 2000; ++t) {
    const int b = (int)(rng() % B), c = (int)(rng() % H);
    const int so = c >> 6, n = c & 63;
    double ref = bias[c];
    for (int e = fptr[so]; e < fptr[so + 1]; ++e) {
      const int si = fidx[e].x, k = fidx[e].y;
      for (int kk = 0; kk < 64; ++kk)
        ref += (double)wb[(size_t)k * 4096 + n * 64 + kk] * x[(size_t)b * H + si * 64 + kk];
    }
    const int rt = b >> 5, g = n >> 3, hh = (n >> 2) & 1, s = n & 3, lane = (b & 31) + 32 * hh;
    const double got = yt[(((size_t)rt * S + so) * 8 + g) * 256 + lane * 4 + s];
    maxerr = std::max(maxerr, std::fabs(got - ref));
  }
  std::printf("max |err| vs fp64 on 2000 samples: %.3e\n", maxerr);
  static hipEvent_t e0, e1;
  if (!e0) { CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); }
  const double flop = 2.0 * 4096.0 * nblk * B;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) run();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    std::printf("kernel %d: %8.1f us  %6.1f TFLOP/s (%.1f%% of 157.3)\n", kern, ms * 1e3,
                flop / (ms * 1e-3) / 1e12, 100.0 * flop / (ms * 1e-3) / 1e12 / 157.3);
  }
  }
  return 0;
}
