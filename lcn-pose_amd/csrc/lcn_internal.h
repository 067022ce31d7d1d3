// Internal declarations shared by the kernel translation units and the C-ABI
// host code (lcn_api.cpp).  gfx950 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lcn {

constexpr int kJ = 17;          // joints (models_att.py:512-513)
constexpr int kSlab = 64;       // feature slab = MFMA tile edge; F is a multiple of it
constexpr int kGemmBM = 128;    // batch rows per block-sparse GEMM tile
constexpr int kLiftRows = 64;   // rows per lift-layer tile (BN partial granularity)
constexpr int kEwRows = 256;    // rows per tile of the BN-backward elementwise kernels

// ----------------------------------------------------------------------------
// Block-sparse GEMM (forward z = a.We + b and backward dA = dZ.We^T).
// Output slab `so` of a row tile accumulates X[:, si-slab] . blocks[blk] over
// the (si, blk) list ptr[so]..ptr[so+1].  Blocks are 64x64, [n][k] (k fastest).
// ----------------------------------------------------------------------------
struct GemmArgs {
  const float* X; int ldx;           // A operand source [B][ldx]
  const float* blocks;               // packed blocks
  const int* ptr;                    // [n_out_slabs + 1]
  const int2* idx;                   // (in_slab, block id)
  const float* bias;                 // [n_out_slabs*64] or null
  const float* pro_scale;            // prologue BN scale per input channel, or null (raw)
  const float* pro_shift;
  int spj_in;                        // input slabs per joint (channel = (si % spj)*64 + k)
  float alpha;                       // LeakyReLU slope of the prologue
  float* Y; int ldy;                 // output [B][ldy]
  const float* addsrc;               // Y = acc (+ addsrc) ; may alias Y
  float2* stat;                      // BN partials [row_tiles][ldy] (sum, m2) or null
  int B; int n_out_slabs; int n_row_tiles;
};
void launch_gemm_bs(const GemmArgs& a, hipStream_t s);

// dWe blocks: part[chunk][blk][p][q] = sum_{b in chunk} A[b, si*64+p] * D[b, so*64+q]
struct GemmDwArgs {
  const float* A; int lda;
  const float* D; int ldd;
  const float* pro_scale; const float* pro_shift; int spj_in; float alpha;
  const int2* blk;                   // (si, so) per block
  int nblk;
  int B; int chunk_rows; int nchunks;
  float* part;                       // [nchunks][nblk][4096]
};
void launch_gemm_dw(const GemmDwArgs& a, hipStream_t s);
// sum partials over chunks; write into dense dW [kin][ld] at (si*64+p, so*64+q)
void launch_dw_reduce(const float* part, int nchunks, int nblk, const int2* blk,
                      float* dW, int ld, hipStream_t s);

// ----------------------------------------------------------------------------
// Small-K layers (lift 34->H and the output layer's dX), VALU.
// out[b, s*64+f] = sum_{u,c} small[b, u*C+c] * coef[s][u][c][f] (+ bias)
// ----------------------------------------------------------------------------
struct ExpandArgs {
  const float* small; int lds_small; int C;
  const float* coef;                 // [n_slabs][J][C][64]
  const unsigned* umask;             // [n_slabs] bit u = joint u contributes
  const float* bias;                 // or null
  float* out; int ldo;
  float2* stat;                      // [B/64 tiles][ldo] or null
  int B; int n_slabs;
};
void launch_expand(const ExpandArgs& a, hipStream_t s);

// part[chunk][s][u][c][f] = sum_b big[b, s*64+f] * small[b, u*C+c] for u in umask[s]
struct OuterArgs {
  const float* big; int ldb;
  const float* small; int lds_small; int C;
  const unsigned* umask;
  int B; int chunk_rows; int nchunks; int n_slabs;
  float* part;                       // [nchunks][n_slabs][J*C][64]
};
void launch_outer(const OuterArgs& a, hipStream_t s);
// reduce over chunks and scatter: mode 0 (lift): dW[(u*C+c)][s*64+f], ld = n_slabs*64
//                                 mode 1 (out):  dW[s*64+f][u*C+c],   ld = J*C
void launch_outer_reduce(const float* part, int nchunks, int n_slabs, int C, int mode,
                         float* dW, hipStream_t s);

// Output layer forward + loss + dy (models_att.py:749-773, :356)
struct OutFwdArgs {
  const float* h; int ldh;           // [B][H]
  const float* w4;                   // dense masked W4e [H][51]
  const float* b4;
  const float* x; int in_f;          // [B][J*in_f]
  const float* lab;                  // [B][51] or null
  float* out;                        // [B][51]
  float* dy;                         // [B][51] or null
  double* loss_part;                 // [gridDim] or null
  float dscale;                      // 2 / (B_global * 51)
  int B; int n_in_slabs;
};
void launch_out_fwd(const OutFwdArgs& a, hipStream_t s);

// ----------------------------------------------------------------------------
// BatchNorm (batch statistics), activation, BN backward
// ----------------------------------------------------------------------------
// stats per channel: mean, rstd, scale = gamma*rstd, shift = beta - mean*scale
struct BnStats { float* mean; float* rstd; float* scale; float* shift; };
// phase 0: complete (single GPU); 1: local s1 -> acc[F]; 2: s2 about mean(acc_s1) -> acc2;
// 3: final from acc1/acc2.  count = rows_global * J.
void launch_bn_finalize(const float2* part, int n_row_tiles, int tile_rows, int B, int H, int F,
                        const float* gamma, const float* beta, float eps, double count,
                        double* acc1, double* acc2, int phase, BnStats st, hipStream_t s);
// h = [res +] leaky(scale*z + shift)
void launch_bn_act(const float* z, const float* res, float* h, const float* scale,
                   const float* shift, int F, float alpha, int B, int H, hipStream_t s);
// partial (sum du, sum du*zhat) per [B/256 tile][H]; du = dh * leaky'(u)
void launch_bnback_reduce(const float* dh, const float* z, const float* scale,
                          const float* shift, const float* mean, const float* rstd, int F,
                          float alpha, int batch_norm, int B, int H, float2* part, hipStream_t s);
// phase 0 complete; 1 local sums -> acc (2F doubles); 2 finish from acc.
// writes dgamma/dbeta (into the raw-grad buffer) and c1,c2,c3
void launch_bnback_finalize(const float2* part, int n_tiles, int H, int F, double count,
                            const float* gamma, const float* mean, const float* rstd,
                            double* acc, int phase, float* dgamma, float* dbeta, float* c123,
                            hipStream_t s);
// dz = c1*du + c2 + c3*z ; per-tile column sums of dz -> bpart[tile][H]
void launch_bnback_apply(const float* dh, const float* z, const float* scale,
                         const float* shift, const float* c123, int F, float alpha,
                         int batch_norm, int B, int H, float* dz, float* bpart, hipStream_t s);
// db[col] = sum_tiles bpart[tile][col]
void launch_colsum(const float* part, int n_tiles, int H, float* out, hipStream_t s);
// per-kEwRows-tile column sums of src[B][ncols] (ncols <= 64) -> part[tiles][ncols]
void launch_colpart(const float* src, int B, int ncols, int ld, float* part, hipStream_t s);
void launch_loss_finalize(const double* part, int n, double* out, hipStream_t s);

// ----------------------------------------------------------------------------
// Parameters: mask, clip_by_norm, masking, packing, gradients, Adam
// ----------------------------------------------------------------------------
struct WLayer {            // one linear layer's weight
  int64_t w_off;           // offset in the flat parameter vector
  int kin, nout, fin, fout;
  int kind;                // 0 lift, 1 hidden, 2 output
  float* dense_e;          // dense masked effective weight (lift/out) or null
  float* coef;             // expand coefficients (lift: fwd; out: bwd-dx) or null
  float* blk_fwd;          // hidden: packed [nblk][q][p]
  float* blk_bwd;          // hidden: packed [nblk][p][q]
  const int2* blk;         // hidden: (si, so) per block (device)
  int nblk;
};
// M = softmax(V,0) (.) C  (LC)  or M = const (EXP); writes M and S
void launch_mask(const float* V, const float* Cmat, int learnable, float* M, float* S,
                 hipStream_t s);
// sum of squares per layer -> norm2[l] (double); denom[l] = max(sqrt, 1) (float)
void launch_wnorm(const float* params, const int64_t* offs, const int64_t* sizes, int nl,
                  double* part, int parts_per_layer, double* norm2, float* denom, int max_norm,
                  hipStream_t s);
// W_e = (W / denom) * M[i,j]; writes the layer's packed / dense / coef forms
void launch_wprep(const float* params, const WLayer& L, const float* M, const float* denom,
                  int layer, hipStream_t s);
// blocksum[l][i][j] = sum_{p,q} dWe * W over joint block (i,j)
void launch_wdot(const float* rg, const float* params, const int64_t* offs, const int* kin,
                 const int* nout, int nl, double* blocksum, hipStream_t s);
// dM, dV (LC) and per-layer clip coefficients coef[l] = (1/denom, c_l)
void launch_maskgrad(const double* blocksum, int nl, const float* M, const float* S,
                     const float* Cmat, int learnable, const float* denom, const double* norm2,
                     int max_norm, float* dV, float* lcoef, hipStream_t s);

// Segment of the flat parameter vector for the fused gradient-finish + Adam.
struct AdamSeg {
  int64_t off, size;
  int kind;                // 0 plain (bias/gamma/beta/mask), 1 weight (clip+mask backward)
  int layer;               // weight: index into lcoef
  int cols, fin, fout;     // weight geometry
  int reg;                 // add regularisation * theta
};
void launch_adam(float* theta, float* m, float* v, const float* rg, float* gout,
                 const AdamSeg* segs, const int64_t* seg_block_start, int nseg,
                 int64_t total_blocks, const float* M, const float* lcoef, float reg,
                 float lr_t, float beta1, float beta2, float eps, int update, hipStream_t s);

}  // namespace lcn
