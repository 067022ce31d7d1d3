// Batched MPJPE / P-MPJPE of evaluate.py on the device (gfx950).
//
// The reference evaluates one frame at a time in a Python loop
// (evaluate.py:53-73): image_to_camera_frame (tools/tools.py:183-194), for
// protocol 2 align_to_gt = procrustes(gt, pred)[1] (tools.py:96-181, 197-202,
// a numpy SVD per frame), then the per-joint distance
// sqrt(sum((pred - gt)^2, axis=1)).  Here one thread owns one frame and does
// all of it in float64 registers:
//
//   * image_to_camera_frame with the reference's operation order (z first,
//     then (u - c) / f, then * z): bit-identical to numpy;
//   * protocol 1 error: ((dx^2 + dy^2) + dz^2) then sqrt, numpy's order for a
//     3-element row: bit-identical;
//   * protocol 2: centred / scale-normalised A = gt, B = pred, the 3x3
//     M = A0^T B0, its SVD by one-sided Jacobi (column rotations of W = M V
//     until the columns are orthogonal; s_i = |w_i|, u_i = w_i / s_i), then
//     R = V U^T and Z = |A| (s1 + s2 + s3) B0 R + mean(A) as procrustes does
//     (scaling=True, reflection='best' -- no reflection fix).  The SVD is a
//     different algorithm from LAPACK's, so protocol 2 agrees with numpy to
//     rounding (~1e-12 mm), not bitwise.
//
// The per-frame work is ~1 kFLOP on 816 B of input: latency/launch-bound on
// the GPU, dominated by the PCIe copies of the host arrays.
#include <cmath>

#include "lcn_internal.h"

namespace lcn {

namespace {

constexpr int kEJ = 17;

// one-sided Jacobi SVD of the 3x3 M (row-major): on return W = M V has
// orthogonal columns, V is orthogonal
__device__ void jacobi_svd3(const double M[9], double W[9], double V[9]) {
  for (int i = 0; i < 9; ++i) { W[i] = M[i]; V[i] = (i % 4 == 0) ? 1.0 : 0.0; }
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = 0.0;
#pragma unroll
    for (int pq = 0; pq < 3; ++pq) {
      const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
      double a = 0.0, b = 0.0, g = 0.0;  // |w_p|^2, |w_q|^2, w_p . w_q
      for (int r = 0; r < 3; ++r) {
        a = fma(W[3 * r + p], W[3 * r + p], a);
        b = fma(W[3 * r + q], W[3 * r + q], b);
        g = fma(W[3 * r + p], W[3 * r + q], g);
      }
      if (g == 0.0) continue;
      const double rel = fabs(g) / sqrt(a * b);
      off = fmax(off, rel);
      if (!(rel > 1e-17)) continue;
      // rotation that zeroes the (p, q) inner product
      const double zeta = (b - a) / (2.0 * g);
      const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
      const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
      for (int r = 0; r < 3; ++r) {
        const double wp = W[3 * r + p], wq = W[3 * r + q];
        W[3 * r + p] = c * wp - s * wq;
        W[3 * r + q] = s * wp + c * wq;
        const double vp = V[3 * r + p], vq = V[3 * r + q];
        V[3 * r + p] = c * vp - s * vq;
        V[3 * r + q] = s * vp + c * vq;
      }
    }
    if (off <= 1e-15) break;
  }
}

__global__ __launch_bounds__(256) void mpjpe_kernel(int64_t n, const double* __restrict__ pred,
                                                    const double* __restrict__ gt,
                                                    const double* __restrict__ box,
                                                    const double* __restrict__ cam,
                                                    const double* __restrict__ root_depth,
                                                    int protocol2, double* __restrict__ err) {
  // numpy rounds every product and sum: no fma contraction outside the
  // explicit fma() calls
#pragma clang fp contract(off)
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  const double* P = pred + f * (kEJ * 3);
  const double* G = gt + f * (kEJ * 3);
  // tools.py:183-194
  const double ratio = (box[4 * f + 2] - box[4 * f + 0] + 1.0) / 2000.0;
  const double rd = root_depth[f];
  const double cx = cam[4 * f + 0], cy = cam[4 * f + 1], fx = cam[4 * f + 2], fy = cam[4 * f + 3];
  double p[kEJ * 3];
  for (int j = 0; j < kEJ; ++j) {
    const double z = P[3 * j + 2] / ratio + rd;
    p[3 * j + 0] = ((P[3 * j + 0] - cx) / fx) * z;
    p[3 * j + 1] = ((P[3 * j + 1] - cy) / fy) * z;
    p[3 * j + 2] = z;
  }
  if (protocol2) {
    // procrustes(A = gt, B = pred): translation, scale, rotation (tools.py:126-172)
    double am[3] = {0.0, 0.0, 0.0}, bm[3] = {0.0, 0.0, 0.0};
    for (int j = 0; j < kEJ; ++j)
      for (int c = 0; c < 3; ++c) { am[c] += G[3 * j + c]; bm[c] += p[3 * j + c]; }
    for (int c = 0; c < 3; ++c) { am[c] /= kEJ; bm[c] /= kEJ; }
    double ssx = 0.0, ssy = 0.0;
    for (int j = 0; j < kEJ; ++j)
      for (int c = 0; c < 3; ++c) {
        const double da = G[3 * j + c] - am[c], db = p[3 * j + c] - bm[c];
        ssx = fma(da, da, ssx);
        ssy = fma(db, db, ssy);
      }
    const double an = sqrt(ssx), bn = sqrt(ssy);
    double M[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // A0^T B0 (normalised)
    for (int j = 0; j < kEJ; ++j) {
      double a0[3], b0[3];
      for (int c = 0; c < 3; ++c) {
        a0[c] = (G[3 * j + c] - am[c]) / an;
        b0[c] = (p[3 * j + c] - bm[c]) / bn;
      }
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) M[3 * r + c] = fma(a0[r], b0[c], M[3 * r + c]);
    }
    double W[9], V[9];
    jacobi_svd3(M, W, V);
    double s[3], U[9];
    for (int c = 0; c < 3; ++c) {
      s[c] = sqrt(W[c] * W[c] + W[3 + c] * W[3 + c] + W[6 + c] * W[6 + c]);
      for (int r = 0; r < 3; ++r) U[3 * r + c] = s[c] > 0.0 ? W[3 * r + c] / s[c] : 0.0;
    }
    // rank-deficient M: complete U to an orthonormal basis (the missing
    // column carries s = 0 and only fixes the sign convention of R)
    for (int c = 0; c < 3; ++c) {
      if (s[c] > 0.0) continue;
      const int c1 = (c + 1) % 3, c2 = (c + 2) % 3;
      U[c] = U[3 + c1] * U[6 + c2] - U[6 + c1] * U[3 + c2];
      U[3 + c] = U[6 + c1] * U[c2] - U[c1] * U[6 + c2];
      U[6 + c] = U[c1] * U[3 + c2] - U[3 + c1] * U[c2];
    }
    double R[9];  // R = V U^T
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        R[3 * r + c] = V[3 * r + 0] * U[3 * c + 0] + V[3 * r + 1] * U[3 * c + 1] + V[3 * r + 2] * U[3 * c + 2];
    const double k = an * (s[0] + s[1] + s[2]);
    for (int j = 0; j < kEJ; ++j) {
      double b0[3];
      for (int c = 0; c < 3; ++c) b0[c] = (p[3 * j + c] - bm[c]) / bn;
      for (int c = 0; c < 3; ++c)
        p[3 * j + c] = k * (b0[0] * R[c] + b0[1] * R[3 + c] + b0[2] * R[6 + c]) + am[c];
    }
  }
  // evaluate.py:61, np.square(pred - gt).sum(axis=1) (a 3-element row is
  // summed left to right) then np.sqrt
  for (int j = 0; j < kEJ; ++j) {
    const double dx = p[3 * j] - G[3 * j], dy = p[3 * j + 1] - G[3 * j + 1], dz = p[3 * j + 2] - G[3 * j + 2];
    err[f * kEJ + j] = sqrt((dx * dx + dy * dy) + dz * dz);
  }
}

}  // namespace

void launch_mpjpe(int64_t n, const double* pred, const double* gt, const double* box, const double* cam,
                  const double* root_depth, int protocol2, double* err, hipStream_t s) {
  const int64_t grid = (n + 127) / 128;
  hipLaunchKernelGGL(mpjpe_kernel, dim3((unsigned)grid), dim3(128), 0, s, n, pred, gt, box, cam, root_depth,
                     protocol2, err);
}

}  // namespace lcn

// ---------------------------------------------------------------------------
// lcn_eval_mpjpe_static: lcn_eval_mpjpe for callers that must not allocate.
//
// lcn_eval_mpjpe stages the host arrays in device buffers it allocates (and
// frees) per call, on a stream it creates.  This variant stages them in a
// fixed array of the code object instead -- `scratch`, one copy per GPU, held
// until the process ends -- and uses the null stream: no hipMalloc, hipFree or
// stream creation, at the price of a frame limit (kStaticMaxFrames per call).
// Every call on a GPU shares that GPU's array: overlapping calls on one GPU
// race (serialise them); nothing in it has to start at zero, each call
// overwrites the part it reads.
// ---------------------------------------------------------------------------
#include <mutex>
#include <string>

#include "../../include/lcn.h"

namespace {

constexpr int64_t kStaticMaxFrames = LCN_EVAL_STATIC_MAX_FRAMES;
// per frame: pred 51 + gt 51 + box 4 + cam 4 + root_depth 1 + err 17 doubles
constexpr int64_t kStaticDoublesPerFrame = 51 + 51 + 4 + 4 + 1 + 17;
constexpr size_t kStaticBytes = (size_t)kStaticMaxFrames * kStaticDoublesPerFrame * sizeof(double);

// In host code this name is only a handle for hipGetSymbolAddress: the
// device address of each GPU's copy is looked up once and kept in
// g_static_ptr; host code passes that pointer, never the array.
static __device__ __align__(256) unsigned char scratch[kStaticBytes];

constexpr int kMaxDevices = 64;
std::mutex g_static_mu;
double* g_static_ptr[kMaxDevices];      // per device, null until looked up
// errors are reported like lcn_eval_mpjpe's: lcn_last_error(NULL)
struct StaticError {
  StaticError& operator=(const std::string& m) { lcn::set_global_error(m); return *this; }
  void clear() { lcn::set_global_error(""); }
} g_static_error;

// the device address of `device`'s copy of the scratch array (device current)
int static_scratch(int device, double** out) {
  std::lock_guard<std::mutex> lock(g_static_mu);
  if (!g_static_ptr[device]) {
    void* p = nullptr;
    const hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(scratch));
    if (e != hipSuccess || !p) {
      g_static_error = std::string("lcn_eval_mpjpe_static: hipGetSymbolAddress: ") + hipGetErrorString(e);
      return LCN_E_HIP;
    }
    g_static_ptr[device] = (double*)p;
  }
  *out = g_static_ptr[device];
  return LCN_OK;
}

}  // namespace

extern "C" int lcn_eval_mpjpe_static(int32_t device, int64_t n, const double* pred, const double* gt,
                                     const double* box, const double* cam, const double* root_depth,
                                     int32_t protocol2, double* err) {
  g_static_error.clear();
  if (device < 0 || device >= kMaxDevices) {
    g_static_error = "lcn_eval_mpjpe_static: device must be in [0, 64)";
    return LCN_E_ARG;
  }
  if (n < 0 || (n > 0 && (!pred || !gt || !box || !cam || !root_depth || !err))) {
    g_static_error = "lcn_eval_mpjpe_static: null argument or negative frame count";
    return LCN_E_ARG;
  }
  if (n > kStaticMaxFrames) {
    g_static_error = "lcn_eval_mpjpe_static: " + std::to_string(n) + " frames exceed the static limit of " +
                     std::to_string(kStaticMaxFrames) + " per call (split the frames, or use lcn_eval_mpjpe)";
    return LCN_E_ARG;
  }
  if (n == 0) return LCN_OK;
  auto fail = [](const char* what, hipError_t e) {
    g_static_error = std::string("lcn_eval_mpjpe_static: ") + what + ": " + hipGetErrorString(e);
    return LCN_E_HIP;
  };
  hipError_t e;
  if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
  double* base = nullptr;
  const int rc = static_scratch(device, &base);
  if (rc != LCN_OK) return rc;
  // sub-arrays at fixed offsets (sized for the frame limit; all multiples of 256 B)
  double* d_pred = base;
  double* d_gt = d_pred + kStaticMaxFrames * 51;
  double* d_box = d_gt + kStaticMaxFrames * 51;
  double* d_cam = d_box + kStaticMaxFrames * 4;
  double* d_root = d_cam + kStaticMaxFrames * 4;
  double* d_err = d_root + kStaticMaxFrames;
  const size_t f = (size_t)n * sizeof(double);
  if ((e = hipMemcpy(d_pred, pred, f * 51, hipMemcpyHostToDevice)) != hipSuccess) return fail("copy pred", e);
  if ((e = hipMemcpy(d_gt, gt, f * 51, hipMemcpyHostToDevice)) != hipSuccess) return fail("copy gt", e);
  if ((e = hipMemcpy(d_box, box, f * 4, hipMemcpyHostToDevice)) != hipSuccess) return fail("copy box", e);
  if ((e = hipMemcpy(d_cam, cam, f * 4, hipMemcpyHostToDevice)) != hipSuccess) return fail("copy cam", e);
  if ((e = hipMemcpy(d_root, root_depth, f, hipMemcpyHostToDevice)) != hipSuccess) return fail("copy root_depth", e);
  lcn::launch_mpjpe(n, d_pred, d_gt, d_box, d_cam, d_root, protocol2 ? 1 : 0, d_err, nullptr);
  if ((e = hipGetLastError()) != hipSuccess) return fail("launch", e);
  // the blocking copy on the null stream waits for the kernel
  if ((e = hipMemcpy(err, d_err, f * lcn::kJ, hipMemcpyDeviceToHost)) != hipSuccess) return fail("copy out", e);
  return LCN_OK;
}
