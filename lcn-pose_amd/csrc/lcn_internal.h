// Internal declarations shared by the kernel translation units and the C-ABI
// host code (lcn_api.cpp).  gfx950 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lcn {

constexpr int kJ = 17;          // joints (models_att.py:512-513)
constexpr int kSlab = 64;       // feature slab = MFMA tile edge; F is a multiple of it
constexpr int kGemmBM = 128;    // batch rows per block-sparse GEMM tile
constexpr int kMinTileRows = 64;  // smallest GEMM row tile (sizes the BN partial buffers)
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
  int variant;                       // tile / pipeline variant (kernels_gemm.hip)
};
void launch_gemm_bs(const GemmArgs& a, hipStream_t s);
int gemm_bs_rows(int variant);       // batch rows per workgroup tile of a variant

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
// sum partials over chunks; write into dense dW [rows][ld] at (si*64+p, so*64+q),
// dropping rows >= rows_valid / columns >= cols_valid (padding of thin layers)
void launch_dw_reduce(const float* part, int nchunks, int nblk, const int2* blk,
                      float* dW, int ld, int rows_valid, int cols_valid, hipStream_t s);

// ----------------------------------------------------------------------------
// The thin layers run on the same MFMA kernels with the narrow side padded to
// one 64-wide slab: the lift's input x [B][17*in_F] lives in a [B][64] buffer
// (K = 34 -> 64) and the output layer's 51 columns in [B][64] buffers.
// ----------------------------------------------------------------------------
// y = h . W4e from the GEMM; out[b, 3j+c] = (c < 2 ? x[b, in_f*j+c] : 0) + (y + b4);
// loss partials and dy = dscale * (out - lab) (padded [B][64]) (models_att.py:765-773, :356)
struct OutAsmArgs {
  const float* y;                    // [B][64] (51 used)
  const float* b4;                   // [51]
  const float* x; int in_f;          // x padded [B][64]
  const float* lab;                  // [B][51] or null
  float* out;                        // [B][51]
  float* dy;                         // [B][64] or null
  double* loss_part;                 // [gridDim] or null
  float dscale;                      // 2 / (B_global * 51)
  int B;
};
void launch_out_assemble(const OutAsmArgs& a, int grid, hipStream_t s);

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
  // packed 64x64 blocks of W_e, K-contiguous ([n][k]) for the MFMA kernels:
  //   hidden: blk_fwd [nblk][q][p], blk_bwd [nblk][p][q]
  //   lift:   blk_fwd [nslab][f][k = u*in_F + c] (k >= 17*in_F zero)
  //   output: blk_fwd [nslab][c'][p], blk_bwd [nslab][p][c'] (c' >= 51 zero)
  float* blk_fwd;
  float* blk_bwd;
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
