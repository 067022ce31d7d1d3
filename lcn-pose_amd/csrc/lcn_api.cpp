// liblcn.so host side: the C ABI of include/lcn.h, device memory plan and the
// per-step kernel schedule that replaces the reference's TF graph + Session.
//
//   forward  (cgcnn._inference_lcn, models_att.py:707-775)
//   loss     (base_model.loss, :352-380)
//   backward (optimizer.compute_gradients, :408) + Adam (:404-409)
//
// One HIP stream per handle; every launch is stream-ordered, the host only
// synchronises when a result is copied back.  After lcn_comm_init (one process per
// GPU) the data-parallel exchanges are RCCL all-reduces on the same stream:
// SyncBN statistics (the reference BN always uses whole-batch statistics) and
// one all-reduce of the raw gradient vector per step.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lcn.h"
#include "lcn_internal.h"

using namespace lcn;

namespace {

thread_local std::string g_create_error;

struct ParamSpec {
  std::string name;
  int64_t off, rows, cols;
};

struct Timer {
  std::vector<hipEvent_t> ev;  // start/stop pairs
  int64_t launches = 0;
  double flops = 0, ms = 0;
};

struct Handle {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;

  // configuration
  int inF = 2, F = 64, L = 3, H = 0, spj = 1, nslab = 0, nl = 0, nbn = 0;
  int learnable = 1, residual = 1, batch_norm = 1, max_norm = 1;
  float eps = 1e-3f, alpha = 0.2f, reg = 0.f, lr0 = 1e-3f, decay_rate = 0.96f;
  float b1 = 0.9f, b2 = 0.999f, adam_eps = 1e-8f;
  int64_t decay_steps = 32000, Bmax = 0;
  std::vector<float> Cmat;  // host copy [17*17]

  // parameters / optimiser
  int64_t P = 0;
  std::vector<ParamSpec> specs;
  float *theta = nullptr, *m = nullptr, *v = nullptr, *rg = nullptr, *gout = nullptr;
  int64_t global_step = 0;
  float b1p = 0.9f, b2p = 0.999f;
  int grads_valid = 0;

  // layers
  std::vector<WLayer> wl;
  std::vector<int64_t> b_off, gamma_off, beta_off;  // per linear layer (-1 if none)
  int64_t mask_off = -1;

  // block structure of the hidden layers (64-granular slabs)
  int nblk = 0;
  int *fwd_ptr = nullptr, *bwd_ptr = nullptr;
  int *fwd_order = nullptr, *bwd_order = nullptr;   // output slabs by falling list length
  // pairs of output slabs of the hidden layers' forward / backward-data GEMMs (PairPlan)
  struct PairDev { int4* pairs = nullptr; int4* ment = nullptr; int* order = nullptr; int n = 0; };
  PairDev fwd_pair, bwd_pair;
  int2 *fwd_idx = nullptr, *bwd_idx = nullptr, *blk = nullptr;
  int *thin_ptr = nullptr, *out_ptr = nullptr;                  // thin layers (padded slab)
  int2 *thin_idx = nullptr, *out_idx = nullptr, *lift_blk = nullptr, *out_blk = nullptr;

  // mask / norms
  float *Md = nullptr, *Sd = nullptr, *Cd = nullptr, *denom = nullptr, *lcoef = nullptr;
  double *norm_part = nullptr, *norm2 = nullptr, *blocksum = nullptr;
  WPrepHidden* wprep_items = nullptr;   // the hidden layers, for the one-launch weight prep
  int64_t *w_offs = nullptr, *w_sizes = nullptr;
  int *w_kin = nullptr, *w_nout = nullptr;
  int norm_ppl = 256;

  // activations
  // x / y / dy of the thin layers are padded to 64 columns (pads stay zero)
  float *x = nullptr, *lab = nullptr, *out = nullptr, *dy = nullptr, *yout = nullptr;
  float* xin = nullptr;           // host-staged row-major input [Bmax][17*in_F]
  std::vector<float*> Z, Hb;
  // dropout (lcn_set_dropout): rate, TF's scale 1/(1-rate), seed, train-step
  // counter; drop_on while a training step runs; Gb = the dropped inner
  // activation g of each block (materialised only with dropout, for the
  // second GEMM of the block and its weight gradient)
  float drop_rate = 0.f, drop_scale = 1.f;
  uint32_t drop_seed = 0, step_seed = 0;
  uint64_t drop_calls = 0;
  bool drop_on = false;
  std::vector<float*> Gb;
  // DH: gradient w.r.t. a block output h_l; DG: w.r.t. the inner activation g;
  // DZ: dz of a hidden layer, stored by its weight-gradient GEMM
  float *DH = nullptr, *DG = nullptr, *DZ = nullptr;
  // weight-gradient work groups (kernels_gemm.hip): up to 2 blocks sharing an output slab
  struct DwMap { int64_t B; DwPlan plan; int4* dev; int n; };   // workgroup map of a launch (make_dw_wgmap)
  struct DwGroups {
    int4* dev = nullptr; int n = 0;
    bool quad = false;           // groups of four blocks, two int4 a group (gemm_dw4.hip)
    int slots = 0;               // quad: workgroups of that kernel the GPU holds at once
    std::vector<DwMap> maps;     // made on first use per batch size
  };
  DwGroups grp_hidden, grp_lift, grp_out;   // grp_hidden.quad: groups of four blocks (gemm_dw4.hip)
  int dw_slots = 0;               // weight-gradient workgroups the GPU holds at once

  std::vector<BnStats> bn;
  std::vector<double*> zsum;      // per BN layer: column sums of z (bias-gradient term)
  float *ident_scale = nullptr, *ident_shift = nullptr, *ident_c123 = nullptr;
  float* c123 = nullptr;
  float2* stat_part = nullptr;    // GEMM epilogue partials [tiles][H], tiles of stat_rows rows
  int stat_rows = kGemmRows;      // rows per partial of the last GEMM: 128, or 32 (small-batch kernel)
  int small_rt = 0;               // launches of at most this many row tiles use the small-batch GEMM
  double2* colacc = nullptr;      // [kColSplit][H] float64 column sums
  int* bn_ticket = nullptr;       // arrival counter of the fused colreduce + BN finish launches (0 between launches)
  float* dw_part = nullptr;
  size_t dw_cap = 0;              // floats in dw_part (sized for max_batch)
  double *loss_part = nullptr, *loss_sum = nullptr, *acc1 = nullptr, *acc2 = nullptr;
  double* db_part = nullptr;      // [loss_grid][64] column sums of dy per out_assemble workgroup
  int loss_grid = 1;

  // Adam segments
  AdamSeg* segs = nullptr;
  int64_t* seg_start = nullptr;
  int nseg = 0;
  int64_t adam_blocks = 0;

  // last batch
  int64_t lastB = 0;

  // user device buffers
  std::vector<void*> user_bufs;
  std::vector<int64_t> user_bytes;

  // device-resident datasets (lcn_dataset_upload) and the predict scratch
  struct Dataset { void* ptr = nullptr; int dtype = 0; int64_t rows = 0; int cols = 0; };
  std::vector<Dataset> datasets;
  int* idx_dev = nullptr;         // [Bmax] batch indices
  double* pred = nullptr;         // [pred_rows][51] float64 predictions of predict_dataset
  double* pred_out = nullptr;     // [pred_rows][51] undone + averaged
  float* batch_losses = nullptr;  // [loss_cap] per-batch predict losses
  int64_t pred_rows = 0, loss_cap = 0;

  // communication: an RCCL communicator (lcn_comm_init) or a host exchange
  // (lcn_comm_init_host: every all-reduce goes through the caller's function)
  ncclComm_t comm = nullptr;
  lcn_host_allreduce_fn host_ar = nullptr;
  void* host_ctx = nullptr;
  std::vector<char> host_stage;
  int rank = 0, world = 1;
  bool comm_off = false;          // lcn_comm_suspend: calls run rank-locally
  bool loss_pending = false;      // the step's loss sum still has to be all-reduced (rides on the first BN backward)
  double* rows_all = nullptr;     // [world] the ranks' batch rows of the running step
  RowInfo* rowinfo = nullptr;     // global rows / first global row of this rank (device)
  // run the multi-GPU (phase 1 -> all-reduce -> phase 2) BN reductions without
  // a communicator (LCN_FORCE_PHASED=1 at create); with one (lcn_comm_init,
  // any world size) they always run phased
  bool phased = false;


  // instrumentation
  int timing = 0;
  std::string timer_err;  // first failure to create / record a timer event since lcn_set_timing
  // train-step graphs (world 1, no dropout, no timing): the device work of a
  // step captured once per (batch, update, keep_grads) and replayed -- small
  // batches are launch-bound (fit's reference batch is 200)
  struct StepGraph { int64_t B; bool update, keep; hipGraphExec_t exec; };
  std::vector<StepGraph> graphs;
  bool capturing = false;  // a step graph is being captured (no allocation / blocking copy allowed)
  int use_graphs = 0;  // LCN_GRAPHS=1 turns them on (rocprofv3 kernel tracing crashed on graph launches)
  float* lr_dev = nullptr;  // Adam's lr_t of the running step
  Timer timers[LCN_K_NUM];

  std::vector<void*> allocs;
};

}  // namespace
void lcn::set_global_error(const std::string& msg) { g_create_error = msg; }
namespace {

#define HIPC(expr)                                                                   \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) {                                                          \
      h->err = std::string(#expr) + ": " + hipGetErrorString(e_);                    \
      return LCN_E_HIP;                                                              \
    }                                                                                \
  } while (0)

#define NCCLC(expr)                                                                  \
  do {                                                                               \
    ncclResult_t r_ = (expr);                                                        \
    if (r_ != ncclSuccess) {                                                         \
      h->err = std::string(#expr) + ": " + ncclGetErrorString(r_);                   \
      return LCN_E_COMM;                                                             \
    }                                                                                \
  } while (0)

#define CHECK(expr)                                                                  \
  do {                                                                               \
    int rc_ = (expr);                                                                \
    if (rc_ != LCN_OK) return rc_;                                                   \
  } while (0)

template <typename T>
int dalloc(Handle* h, T** p, size_t count) {
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
  if (e != hipSuccess) {
    h->err = "hipMalloc(" + std::to_string(count * sizeof(T)) + " bytes): " + hipGetErrorString(e);
    return LCN_E_NOMEM;
  }
  h->allocs.push_back(q);
  e = hipMemset(q, 0, std::max<size_t>(count, 1) * sizeof(T));
  if (e != hipSuccess) {
    h->err = std::string("hipMemset of a new allocation: ") + hipGetErrorString(e);
    return LCN_E_HIP;
  }
  *p = (T*)q;
  return LCN_OK;
}

template <typename T>
int upload(Handle* h, T** p, const std::vector<T>& src) {
  CHECK(dalloc(h, p, src.size()));
  HIPC(hipMemcpy(*p, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  return LCN_OK;
}

int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

int gemm_pair_mode();

// Pair the blocks of each output slab into weight-gradient work groups
// (so, block0, block1 | -1, rank | count << 8): the group's rank among the
// groups of its output slab and their number -- they all rebuild the same dz
// and take turns storing it (item i is stored by the group of rank i % count).
int upload_dw_groups(Handle* h, const std::vector<int2>& blk, Handle::DwGroups* out, bool try_quads = false) {
  int nso = 0;
  for (const int2& b : blk) nso = std::max(nso, b.y + 1);
  std::vector<int4> g;
  // Four blocks a group where every output slab holds a multiple of four (several
  // slabs per joint; the cfg4 shape: 68): the kernel that shares the staged dz
  // between four blocks (cfg4 shape, 16 384 rows: 5.23 -> 4.98 ms a launch).  Two int4 per
  // group: (so, 4, rank, count), (b0, b1, b2, b3).  LCN_DW_QUAD=0: never.
  bool quads = try_quads && !(std::getenv("LCN_DW_QUAD") && std::atoi(std::getenv("LCN_DW_QUAD")) == 0) &&
               blk.size() < 65536;
  std::vector<std::vector<int>> by_so(nso);
  for (size_t b = 0; b < blk.size(); ++b) by_so[blk[b].y].push_back((int)b);
  for (const auto& ids : by_so) quads = quads && !ids.empty() && ids.size() % 4 == 0;
  if (quads) {
    for (int so = 0; so < nso; ++so) {
      const auto& ids = by_so[so];
      const int count = (int)ids.size() / 4;
      for (int q = 0; q < count; ++q) {
        g.push_back(make_int4(so, 4, q, count));
        g.push_back(make_int4(ids[4 * q], ids[4 * q + 1], ids[4 * q + 2], ids[4 * q + 3]));
      }
    }
    out->n = (int)g.size() / 2;
    out->quad = true;
    out->slots = gemm_dw4_resident_slots();
    if (out->slots <= 0) { h->err = "occupancy query of the weight-gradient kernel failed"; return LCN_E_HIP; }
    return upload(h, &out->dev, g);
  }
  for (int so = 0; so < nso; ++so) {
    std::vector<int> ids;
    for (size_t b = 0; b < blk.size(); ++b)
      if (blk[b].y == so) ids.push_back((int)b);
    for (size_t i = 0; i < ids.size(); i += 2)
      g.push_back(make_int4(so, ids[i], i + 1 < ids.size() ? ids[i + 1] : -1, (int)(i / 2) | ((int)((ids.size() + 1) / 2) << 8)));
  }
  out->n = (int)g.size();
  return upload(h, &out->dev, g);
}

// batch chunks of a weight-gradient launch (partials per block = chunks);
// LCN_DW_ROWS / LCN_DW_MAXCH / LCN_DW_MINCH override the block-rows budget and the limits (tuning runs)
int dw_chunks(int nblk, int64_t B) {
  static const int budget = std::getenv("LCN_DW_ROWS") ? std::atoi(std::getenv("LCN_DW_ROWS")) : 5600;
  static const int cap = std::getenv("LCN_DW_MAXCH") ? std::atoi(std::getenv("LCN_DW_MAXCH")) : 64;
  // At least 16 chunks, and chunks of at most 2048 rows: with many blocks
  // (F >= 128: 4 624 at the cfg4 shape) one chunk per block leaves 2.3 rounds of
  // long workgroups and a third of the last round idle (cfg4 shape, 16 384 rows
  // per GPU, same box: 1 / 4 / 8 / 16 chunks 6.05 / 5.61 / 5.85 / 5.37 ms per
  // launch; 24 / 32 / 64 slower again)
  static const int lo = std::getenv("LCN_DW_MINCH") ? std::atoi(std::getenv("LCN_DW_MINCH")) : 16;
  const int by_rows = (int)std::min<int64_t>(cap, B / 2048);
  return std::max(std::max(lo, by_rows), std::min(cap, budget / std::max(1, nblk)));
}

// How a weight-gradient launch over the groups g (nblk blocks) splits B rows
// (lcn_internal.h DwPlan): XCD-strided items in rounds of falling size when
// the groups are few, dw_chunks contiguous chunks otherwise; at most 128
// partials a block.  LCN_DW_SLOTS overrides the resident-slot count (0: always
// contiguous chunks).
DwPlan dw_plan(const Handle* h, const Handle::DwGroups& g, int nblk, int64_t B) {
  static const int slots_env = std::getenv("LCN_DW_SLOTS") ? std::atoi(std::getenv("LCN_DW_SLOTS")) : -1;
  return make_dw_plan(B, g.n, slots_env >= 0 ? slots_env : (g.slots > 0 ? g.slots : h->dw_slots), dw_chunks(nblk, B), 128);
}

// Launches of at most this many 32-row tiles run the small-batch kernel, which
// splits every slab list over the four waves of a workgroup: measured faster
// up to batch 2560 (0.92 -> 0.57 ms per step at batch 200, 1.24 -> 0.89 ms at
// 1024, 1.40 -> 1.29 ms at 2048, 1.49 -> 1.44 ms at 2560), slower from 3072 on
// (1.56 -> 1.61 ms).  LCN_SMALL_RT overrides, 0 = never.
int small_row_tiles() {  // read when a handle is created
  return std::getenv("LCN_SMALL_RT") ? std::atoi(std::getenv("LCN_SMALL_RT")) : 80;
}

// ---------------------------------------------------------------------------
// construction
// ---------------------------------------------------------------------------
int build(Handle* h, const lcn_config* c) {
  if (const char* fp = std::getenv("LCN_FORCE_PHASED")) h->phased = std::atoi(fp) != 0;
  h->small_rt = small_row_tiles();
  h->inF = c->in_f;
  h->F = c->f;
  h->L = c->num_layers;
  h->H = kJ * h->F;
  h->spj = h->F / kSlab;
  h->nslab = kJ * h->spj;
  h->nl = 2 * h->L + 2;
  h->learnable = c->mask_type == LCN_MASK_LOCALLY_CONNECTED;
  h->residual = c->residual;
  h->batch_norm = c->batch_norm;
  h->max_norm = c->max_norm;
  h->eps = c->bn_eps;
  h->alpha = c->leaky_alpha;
  h->reg = c->regularization;
  h->lr0 = c->learning_rate;
  h->decay_rate = c->decay_rate;
  h->decay_steps = c->decay_steps;
  h->b1 = c->beta1;
  h->b2 = c->beta2;
  h->adam_eps = c->adam_eps;
  h->b1p = h->b1;
  h->b2p = h->b2;
  h->Bmax = c->max_batch;
  h->Cmat.assign(c->mask_matrix, c->mask_matrix + kJ * kJ);
  const int H = h->H, F = h->F, inF = h->inF, nl = h->nl;

  // ---- parameter layout (TF variable creation order) ----
  int64_t off = 0;
  auto add = [&](const std::string& n, int64_t r, int64_t cc) {
    h->specs.push_back({n, off, r, cc});
    off += r * cc;
    return off - r * cc;
  };
  if (h->learnable) h->mask_off = add("mask", kJ, kJ);
  h->b_off.assign(nl, -1);
  h->gamma_off.assign(nl, -1);
  h->beta_off.assign(nl, -1);
  h->wl.resize(nl);
  auto layer = [&](int k, const std::string& wn, const std::string& bnm, const std::string& bnp,
                   int fin, int fout, int kind) {
    WLayer& Lr = h->wl[k];
    std::memset(&Lr, 0, sizeof(Lr));
    Lr.kin = kJ * fin;
    Lr.nout = kJ * fout;
    Lr.fin = fin;
    Lr.fout = fout;
    Lr.kind = kind;
    Lr.w_off = add(wn, Lr.kin, Lr.nout);
    h->b_off[k] = add(bnm, 1, Lr.nout);
    if (!bnp.empty() && h->batch_norm) {
      h->gamma_off[k] = add(bnp + "_gamma", 1, F);
      h->beta_off[k] = add(bnp + "_beta", 1, F);
    }
  };
  layer(0, "w1", "b1", "bn0", inF, F, 0);
  for (int l = 0; l < h->L; ++l) {
    const std::string s = std::to_string(l);
    layer(2 * l + 1, "w2_" + s, "b2_" + s, "bn1" + s, F, F, 1);
    layer(2 * l + 2, "w3_" + s, "b3_" + s, "bn2" + s, F, F, 1);
  }
  layer(nl - 1, "w4", "b4", "", F, 3, 2);
  h->P = off;

  CHECK(dalloc(h, &h->theta, h->P));
  CHECK(dalloc(h, &h->m, h->P));
  CHECK(dalloc(h, &h->v, h->P));
  CHECK(dalloc(h, &h->rg, h->P));
  CHECK(dalloc(h, &h->gout, h->P));

  // ---- block structure (joint support S[i][j] at 64-feature granularity) ----
  auto sup = [&](int i, int j) { return h->Cmat[i * kJ + j] != 0.f; };
  std::vector<int2> blk;
  std::vector<int> bid(h->nslab * h->nslab, -1);
  for (int si = 0; si < h->nslab; ++si)
    for (int so = 0; so < h->nslab; ++so)
      if (sup(si / h->spj, so / h->spj)) {
        bid[si * h->nslab + so] = (int)blk.size();
        blk.push_back(make_int2(si, so));
      }
  h->nblk = (int)blk.size();
  std::vector<int> fptr(1, 0), bptr(1, 0);
  std::vector<int2> fidx, bidx;
  for (int so = 0; so < h->nslab; ++so) {
    for (int si = 0; si < h->nslab; ++si)
      if (bid[si * h->nslab + so] >= 0) fidx.push_back(make_int2(si, bid[si * h->nslab + so]));
    fptr.push_back((int)fidx.size());
  }
  for (int si = 0; si < h->nslab; ++si) {
    for (int so = 0; so < h->nslab; ++so)
      if (bid[si * h->nslab + so] >= 0) bidx.push_back(make_int2(so, bid[si * h->nslab + so]));
    bptr.push_back((int)bidx.size());
  }
  CHECK(upload(h, &h->blk, blk));
  CHECK(upload_dw_groups(h, blk, &h->grp_hidden, true));
  CHECK(upload(h, &h->fwd_ptr, fptr));
  CHECK(upload(h, &h->bwd_ptr, bptr));
  CHECK(upload(h, &h->fwd_idx, fidx));
  CHECK(upload(h, &h->bwd_idx, bidx));
  // tail schedule of the block-sparse GEMMs: output slabs, longest list first
  auto by_length = [&](const std::vector<int>& ptr) {
    std::vector<int> o(h->nslab);
    for (int i = 0; i < h->nslab; ++i) o[i] = i;
    std::stable_sort(o.begin(), o.end(), [&](int x, int y) { return ptr[x + 1] - ptr[x] > ptr[y + 1] - ptr[y]; });
    return o;
  };
  CHECK(upload(h, &h->fwd_order, by_length(fptr)));
  CHECK(upload(h, &h->bwd_order, by_length(bptr)));
  // Two output slabs per workgroup pay where a joint has several slabs (their
  // lists are identical: half the activation loads; the cfg4 shape's forward
  // GEMM 4.57 -> 4.43 ms).  With one slab per joint (41 % of the loads saved at
  // knn 3) the shorter loop is offset by two epilogues in a row at three
  // workgroups per CU: forward +-0, backward-data +2.5 % in the cfg3 step.
  if (const int pm = gemm_pair_mode(); pm == 1 || (pm < 0 && h->spj > 1)) {
    auto up = [&](const std::vector<int>& ptr, const std::vector<int2>& idx, Handle::PairDev* d) {
      const PairPlan pp = make_pair_plan(ptr, idx, h->nslab);
      CHECK(upload(h, &d->pairs, pp.pairs));
      CHECK(upload(h, &d->ment, pp.ment));
      CHECK(upload(h, &d->order, pp.order));
      d->n = (int)pp.pairs.size();
      return (int)LCN_OK;
    };
    CHECK(up(fptr, fidx, &h->fwd_pair));
    CHECK(up(bptr, bidx, &h->bwd_pair));
  }
  for (int so = 0; so < h->nslab; ++so)
    if (fptr[so + 1] == fptr[so]) {
      h->err = "output joint " + std::to_string(so / h->spj) + " has no input joint in the mask";
      return LCN_E_ARG;
    }
  // Thin layers as one padded 64-wide slab on the narrow side:
  //   lift:  input slab 0 (x padded to 64) -> every output slab so, block so
  //   out:   every input slab si -> output slab 0 (51 of 64 columns), block si
  //   out^T: input slab 0 (dy padded) -> every output slab so, block so
  std::vector<int> tptr, optr{0, h->nslab};
  std::vector<int2> tidx, oidx, lblk, oblk;
  for (int s = 0; s <= h->nslab; ++s) tptr.push_back(s);
  for (int s = 0; s < h->nslab; ++s) {
    tidx.push_back(make_int2(0, s));
    oidx.push_back(make_int2(s, s));
    lblk.push_back(make_int2(0, s));
    oblk.push_back(make_int2(s, 0));
  }
  CHECK(upload(h, &h->thin_ptr, tptr));
  CHECK(upload(h, &h->thin_idx, tidx));
  CHECK(upload(h, &h->out_ptr, optr));
  CHECK(upload(h, &h->out_idx, oidx));
  CHECK(upload(h, &h->lift_blk, lblk));
  CHECK(upload(h, &h->out_blk, oblk));
  CHECK(upload_dw_groups(h, lblk, &h->grp_lift));
  CHECK(upload_dw_groups(h, oblk, &h->grp_out));

  // ---- per-layer weight forms ----
  for (int k = 0; k < nl; ++k) {
    WLayer& Lr = h->wl[k];
    if (Lr.kind == 1) {
      CHECK(dalloc(h, &Lr.blk_fwd, (size_t)h->nblk * 4096));
      CHECK(dalloc(h, &Lr.blk_bwd, (size_t)h->nblk * 4096));
      Lr.blk = h->blk;
      Lr.nblk = h->nblk;
    } else if (Lr.kind == 0) {
      CHECK(dalloc(h, &Lr.blk_fwd, (size_t)h->nslab * 4096));
    } else {
      CHECK(dalloc(h, &Lr.blk_fwd, (size_t)h->nslab * 4096));
      CHECK(dalloc(h, &Lr.blk_bwd, (size_t)h->nslab * 4096));
    }
  }
  {
    std::vector<WPrepHidden> items;
    for (int k = 0; k < nl; ++k)
      if (h->wl[k].kind == 1) items.push_back(WPrepHidden{h->wl[k].w_off, h->wl[k].blk_fwd, h->wl[k].blk_bwd, k});
    CHECK(upload(h, &h->wprep_items, items));
  }
  // norms: entries [0, nl) are the weights (clip_by_norm), [nl, 2nl) the biases
  // (only for the l2 regularisation term of the reported loss)
  std::vector<int64_t> wo(2 * nl), ws(2 * nl);
  std::vector<int> wk(nl), wn(nl);
  for (int k = 0; k < nl; ++k) {
    wo[k] = h->wl[k].w_off;
    ws[k] = (int64_t)h->wl[k].kin * h->wl[k].nout;
    wo[nl + k] = h->b_off[k];
    ws[nl + k] = h->wl[k].nout;
    wk[k] = h->wl[k].kin;
    wn[k] = h->wl[k].nout;
  }
  CHECK(upload(h, &h->w_offs, wo));
  CHECK(upload(h, &h->w_sizes, ws));
  CHECK(upload(h, &h->w_kin, wk));
  CHECK(upload(h, &h->w_nout, wn));
  CHECK(upload(h, &h->Cd, h->Cmat));
  CHECK(dalloc(h, &h->Md, kJ * kJ));
  CHECK(dalloc(h, &h->Sd, kJ * kJ));
  CHECK(dalloc(h, &h->denom, nl));
  CHECK(dalloc(h, &h->lcoef, 2 * nl));
  CHECK(dalloc(h, &h->norm_part, (size_t)2 * nl * h->norm_ppl));
  CHECK(dalloc(h, &h->norm2, 2 * nl));
  CHECK(dalloc(h, &h->blocksum, (size_t)nl * kJ * kJ));

  // ---- Adam segments ----
  std::vector<AdamSeg> segs;
  std::vector<int64_t> starts;
  int64_t blocks = 0;
  for (const ParamSpec& ps : h->specs) {
    AdamSeg sg{};
    sg.off = ps.off;
    sg.size = ps.rows * ps.cols;
    sg.kind = 0;
    sg.layer = -1;
    for (int k = 0; k < nl; ++k)
      if (h->wl[k].w_off == ps.off) {
        sg.kind = 1;
        sg.layer = k;
        sg.cols = h->wl[k].nout;
        sg.fin = h->wl[k].fin;
        sg.fout = h->wl[k].fout;
        sg.reg = h->reg != 0.f;
      }
    for (int k = 0; k < nl; ++k)
      if (h->b_off[k] == ps.off) sg.reg = h->reg != 0.f;
    segs.push_back(sg);
    starts.push_back(blocks);
    blocks += cdiv(sg.size, 1024);
  }
  h->nseg = (int)segs.size();
  h->adam_blocks = blocks;
  CHECK(upload(h, &h->segs, segs));
  CHECK(upload(h, &h->seg_start, starts));

  // ---- activations / scratch for Bmax ----
  const int64_t B = h->Bmax;
  // activations in the row-tile layout (lcn_internal.h); x / y / dy of the
  // thin layers are one 64-wide slab
  const size_t t1 = (size_t)tiled_floats(B, 1), tH = (size_t)tiled_floats(B, h->nslab);
  CHECK(dalloc(h, &h->x, t1));
  CHECK(dalloc(h, &h->xin, (size_t)B * kJ * h->inF));
  CHECK(dalloc(h, &h->idx_dev, (size_t)B));
  CHECK(dalloc(h, &h->lab, (size_t)B * 51));
  CHECK(dalloc(h, &h->out, (size_t)B * 51));
  CHECK(dalloc(h, &h->dy, t1));
  CHECK(dalloc(h, &h->yout, t1));
  h->Z.assign(nl - 1, nullptr);
  for (auto& z : h->Z) CHECK(dalloc(h, &z, tH));
  h->Hb.assign(h->L + 1, nullptr);
  for (auto& hb : h->Hb) CHECK(dalloc(h, &hb, tH));
  CHECK(dalloc(h, &h->DH, tH));
  CHECK(dalloc(h, &h->DG, tH));
  CHECK(dalloc(h, &h->DZ, tH));
  CHECK(dalloc(h, &h->lr_dev, 1));
  if (const char* g = std::getenv("LCN_GRAPHS")) h->use_graphs = std::atoi(g) != 0;
  h->zsum.assign(nl - 1, nullptr);
  for (auto& zs : h->zsum) CHECK(dalloc(h, &zs, (size_t)H));
  h->nbn = nl - 1;
  h->bn.resize(h->nbn);
  std::vector<float> ones(F, 1.f), zeros(F, 0.f), ic(3 * F, 0.f);
  for (int f = 0; f < F; ++f) ic[f] = 1.f;
  CHECK(upload(h, &h->ident_scale, ones));
  CHECK(upload(h, &h->ident_shift, zeros));
  CHECK(upload(h, &h->ident_c123, ic));
  for (auto& s : h->bn) {
    if (h->batch_norm) {
      CHECK(dalloc(h, &s.mean, F));
      CHECK(dalloc(h, &s.rstd, F));
      CHECK(dalloc(h, &s.scale, F));
      CHECK(dalloc(h, &s.shift, F));
    } else {
      s.mean = h->ident_shift;
      s.rstd = h->ident_scale;
      s.scale = h->ident_scale;
      s.shift = h->ident_shift;
    }
  }
  CHECK(dalloc(h, &h->c123, 3 * F));
  CHECK(dalloc(h, &h->stat_part,
               (size_t)std::max<int64_t>(cdiv(B, kGemmRows), std::min<int64_t>(cdiv(B, kRT), h->small_rt)) * H));
  CHECK(dalloc(h, &h->colacc, (size_t)kColSplit * H));
  CHECK(dalloc(h, &h->bn_ticket, 1));
  h->loss_grid = (int)std::min<int64_t>(2048, cdiv(B, 4));
  CHECK(dalloc(h, &h->loss_part, (size_t)h->loss_grid));
  CHECK(dalloc(h, &h->db_part, (size_t)h->loss_grid * 64));
  CHECK(dalloc(h, &h->loss_sum, 4));
  CHECK(dalloc(h, &h->acc1, 2 * F));
  CHECK(dalloc(h, &h->acc2, 2 * F));
  CHECK(dalloc(h, &h->rowinfo, 1));
  // chunk partials of the weight gradient, with the launch's own clamp (a chunk
  // holds at least 64 rows): 16 KB per block and chunk -- 92 MB at the cfg3
  // shape (175 blocks, 32 chunks), 1.2 GB at the cfg4 shape with 16 384 rows
  // (4 624 blocks, 16 chunks)
  h->dw_slots = gemm_dw_resident_slots();
  if (h->dw_slots <= 0) { h->err = "occupancy query of the weight-gradient kernel failed"; return LCN_E_HIP; }
  h->dw_cap = (size_t)std::max({(int64_t)dw_plan_slots(dw_plan(h, h->grp_hidden, h->nblk, B)) * h->nblk,
                                (int64_t)dw_plan_slots(dw_plan(h, h->grp_lift, h->nslab, B)) * h->nslab,
                                (int64_t)dw_plan_slots(dw_plan(h, h->grp_out, h->nslab, B)) * h->nslab}) * 4096;
  CHECK(dalloc(h, &h->dw_part, h->dw_cap));
  return LCN_OK;
}

// ---------------------------------------------------------------------------
// step pieces
// ---------------------------------------------------------------------------
// several ranks (or a one-rank communicator): the step runs the phased BN
// reductions and every exchange below
bool has_comm(const Handle* h) { return h->comm != nullptr || h->host_ar != nullptr; }
bool multi(const Handle* h) { return has_comm(h) && !h->comm_off; }

// In-place all-reduce of a device buffer over the ranks, stream-ordered: RCCL,
// or (host exchange) device -> host, the caller's function, host -> device.
void tstart(Handle* h, int k, hipEvent_t* pair);
void tstop(Handle* h, int k, hipEvent_t* pair, double flops);

int allreduce_untimed(Handle* h, void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op);

int allreduce(Handle* h, void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op = ncclSum) {
  if (h->comm_off) return LCN_OK;  // suspended: the call runs rank-locally (phased reductions included)
  if (!h->comm && !h->host_ar) return LCN_OK;
  hipEvent_t ev[2];
  tstart(h, LCN_K_COMM, ev);
  const int rc = allreduce_untimed(h, buf, count, dt, op);
  tstop(h, LCN_K_COMM, ev, (double)count * (dt == ncclDouble ? 8 : 4));
  return rc;
}

int allreduce_untimed(Handle* h, void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op) {
  if (h->comm) {
    NCCLC(ncclAllReduce(buf, buf, count, dt, op, h->comm, h->stream));
    return LCN_OK;
  }
  const size_t bytes = count * (dt == ncclDouble ? 8 : 4);
  if (h->host_stage.size() < bytes) h->host_stage.resize(bytes);
  HIPC(hipMemcpyAsync(h->host_stage.data(), buf, bytes, hipMemcpyDeviceToHost, h->stream));
  HIPC(hipStreamSynchronize(h->stream));
  const int rc = h->host_ar(h->host_ctx, h->host_stage.data(), (int64_t)count,
                            dt == ncclDouble ? LCN_DTYPE_F64 : LCN_DTYPE_F32, op == ncclMax ? 1 : 0);
  if (rc != 0) {
    h->err = "host all-reduce callback failed (" + std::to_string(rc) + ")";
    return LCN_E_COMM;
  }
  HIPC(hipMemcpyAsync(buf, h->host_stage.data(), bytes, hipMemcpyHostToDevice, h->stream));
  // the staging buffer is reused by the next exchange
  HIPC(hipStreamSynchronize(h->stream));
  return LCN_OK;
}

// The ranks' shards may differ in size: gather every rank's batch rows (an
// all-reduce of a one-hot vector) and derive the global row count and this
// rank's first global row on the device (RowInfo), where the BN finishes, the
// loss scale and the dropout keys read them.
int exchange_rows(Handle* h, int64_t B) {
  if (!multi(h)) return LCN_OK;
  launch_rows_begin(h->rows_all, h->world, h->rank, B, h->stream);
  CHECK(allreduce(h, h->rows_all, (size_t)h->world, ncclDouble));
  launch_rows_finish(h->rows_all, h->world, h->rank, h->rowinfo, h->stream);
  return LCN_OK;
}
// what the kernels take: the device RowInfo with several ranks, else null
// (then the by-value local row count is the global one)
const RowInfo* rinfo(const Handle* h) { return multi(h) ? h->rowinfo : nullptr; }

// lcn_set_timing: 1 = every kernel class, else bit k + 1 selects class k
bool timed(const Handle* h, int k) { return h->timing == 1 || ((h->timing >> (k + 1)) & 1); }

// A launch whose timer events cannot be created runs untimed (pair[0] stays
// null and tstop skips it); the failure is kept for lcn_kernel_timing.
void tstart(Handle* h, int k, hipEvent_t* pair) {
  pair[0] = pair[1] = nullptr;
  if (!timed(h, k)) return;
  // timing-only events: no system-scope fence when they complete
  hipError_t e = hipEventCreateWithFlags(&pair[0], hipEventDisableSystemFence);
  if (e == hipSuccess) {
    e = hipEventCreateWithFlags(&pair[1], hipEventDisableSystemFence);
    if (e != hipSuccess) hipEventDestroy(pair[0]);
  }
  if (e == hipSuccess) e = hipEventRecord(pair[0], h->stream);
  if (e != hipSuccess) {
    h->timer_err = std::string("kernel timer events: ") + hipGetErrorString(e);
    pair[0] = pair[1] = nullptr;
  }
}
void tstop(Handle* h, int k, hipEvent_t* pair, double flops) {
  if (!timed(h, k) || !pair[0]) return;
  hipEventRecord(pair[1], h->stream);
  h->timers[k].ev.push_back(pair[0]);
  h->timers[k].ev.push_back(pair[1]);
  h->timers[k].launches++;
  h->timers[k].flops += flops;
}

// the dropout of BN layer k in the running training step (rate 0 = none)
Dropout drop_of(const Handle* h, int k, int64_t B) {
  Dropout d{};
  d.rate = 0.f;
  d.scale = 1.f;
  if (!h->drop_on) return d;
  d.rate = h->drop_rate;
  d.scale = h->drop_scale;
  d.lseed = fmix32(h->step_seed ^ ((uint32_t)(k + 1) * 0x9e3779b9u));
  d.H = h->H;
  d.row0 = 0;
  d.ri = rinfo(h);
  (void)B;
  return d;
}

int prep_weights(Handle* h) {
  hipStream_t s = h->stream;
  launch_mask(h->learnable ? h->theta + h->mask_off : nullptr, h->Cd, h->learnable, h->Md, h->Sd, s);
  launch_wnorm(h->theta, h->w_offs, h->w_sizes, 2 * h->nl, h->norm_part, h->norm_ppl, h->norm2,
               h->denom, h->max_norm, s);
  launch_wprep_hidden(h->theta, h->wprep_items, 2 * h->L, h->H, h->blk, h->nblk, h->spj, h->Md, h->denom, s);
  launch_wprep(h->theta, h->wl[0], h->Md, h->denom, 0, s);
  launch_wprep(h->theta, h->wl[h->nl - 1], h->Md, h->denom, h->nl - 1, s);
  return LCN_OK;
}

// The last GEMM's epilogue partials for the BN finish kernels: with at most 8
// tiles (batch <= 256 behind the small-batch GEMM, <= 1024 otherwise) the
// finish sums them itself -- a colreduce launch costs ~4 us, as much as the
// whole reduction then; with more tiles the one finishing workgroup's serial
// walk over them is slower than the extra launch (measured at 32 and 64 tiles)
TilePartials tile_partials(const Handle* h, int B) {
  const int n_tiles = (int)cdiv(B, h->stat_rows);
  if (n_tiles > 8) return TilePartials{nullptr, 0, 0, 0};
  return TilePartials{h->stat_part, n_tiles, h->stat_rows, B};
}

// BN statistics of BN layer k from the EPI_BNFWD partials its GEMM wrote
// (one SyncBN all-reduce of 2F doubles with several GPUs); also keeps the
// column sums of z for the bias gradient of the backward
int bn_stats(Handle* h, int k, int B) {
  if (!h->batch_norm) return LCN_OK;
  hipStream_t s = h->stream;
  const double rows = (double)B;
  const RowInfo* ri = rinfo(h);
  const float* gamma = h->theta + h->gamma_off[k];
  const float* beta = h->theta + h->beta_off[k];
  const TilePartials tp = tile_partials(h, B);
  const BnRider none{};
  // many tiles: their column reduce and the finish (phase 0 / 1) are one launch
  const int n_tiles = (int)cdiv(B, h->stat_rows);
  if (!h->phased && !multi(h)) {
    if (!tp.part)
      launch_colreduce_bn_fwd(h->stat_part, n_tiles, h->stat_rows, B, h->colacc, h->bn_ticket, h->H, h->F, 0,
                              rows, ri, gamma, beta, h->eps, h->acc1, h->bn[k], h->zsum[k], none, s);
    else
      launch_bn_fwd_finalize(h->colacc, tp, h->H, h->F, 0, rows, ri, gamma, beta, h->eps, h->acc1, h->bn[k],
                             h->zsum[k], none, s);
    return LCN_OK;
  }
  // several ranks: BN layer 0's all-reduce also carries the ranks' batch rows
  // (the first exchange of a step; nothing before its finish reads RowInfo)
  BnRider rider{};
  if (multi(h) && k == 0) {
    rider.kind = kRideRows;
    rider.world = h->world;
    rider.rank = h->rank;
    rider.b_local = rows;
    rider.ri_out = h->rowinfo;
  }
  if (!tp.part)
    launch_colreduce_bn_fwd(h->stat_part, n_tiles, h->stat_rows, B, h->colacc, h->bn_ticket, h->H, h->F, 1,
                            rows, ri, gamma, beta, h->eps, h->acc1, h->bn[k], h->zsum[k], rider, s);
  else
    launch_bn_fwd_finalize(h->colacc, tp, h->H, h->F, 1, rows, ri, gamma, beta, h->eps, h->acc1, h->bn[k],
                           h->zsum[k], rider, s);
  CHECK(allreduce(h, h->acc1, 2 * h->F + rider_slots(rider), ncclDouble));
  launch_bn_fwd_finalize(h->colacc, tp, h->H, h->F, 2, rows, ri, gamma, beta, h->eps, h->acc1, h->bn[k],
                         nullptr, rider, s);
  return LCN_OK;
}

// A GEMM operand: a row-tiled tensor of S slabs, read as is (PRO_RAW), through
// BN apply + LeakyReLU of BN layer `layer` (PRO_BNACT: p = z of that layer),
// or as the dz of BN layer `layer` rebuilt from p = dh and its z (PRO_BNBACK).
struct Operand {
  const float* p; int S;
  int mode; int layer;
};
Operand raw(const float* p, int S) { return Operand{p, S, PRO_RAW, -1}; }

// One launch of the block-sparse MFMA GEMM: Y[:, so-slab] = sum over the CSR
// list of X[:, si-slab] . block (+ bias / + addsrc); epilogue partials:
// EPI_BNFWD (BN statistics of Y) or EPI_BNBACK for BN layer `epi_layer`.
// `timer` < 0: not timed.
struct GemmCall {
  Operand X;
  const float* blocks; const int* ptr; const int2* idx; int n_out_slabs;
  const float* bias;
  float* Y; int S_out; const float* addsrc;
  int epi_mode; int epi_layer;
  int timer; double flops_per_row;
  const int* order = nullptr;   // tail schedule (hidden layers); null: natural order
  int k_groups = 0;             // non-zero 8-feature groups of the input slab (the lift), 0 = all
  const Handle::PairDev* pair = nullptr;  // hidden layers: pairs of output slabs, or null
};

// row-tile groups per XCD issued longest-list-first at the end of a launch
// (LCN_GEMM_TAIL overrides, 0 = natural order throughout)
int tail_groups() {
  static const int t = std::getenv("LCN_GEMM_TAIL") ? std::atoi(std::getenv("LCN_GEMM_TAIL")) : 16;
  return t;
}

// two output slabs per workgroup for the hidden layers' large launches
// (gemm_pair.hip): LCN_GEMM_PAIR=1 always, 0 never, unset: where a joint has
// several slabs.  Read at handle creation.
int gemm_pair_mode() {
  const char* e = std::getenv("LCN_GEMM_PAIR");
  return e ? (std::atoi(e) != 0) : -1;
}

int gemm(Handle* h, const GemmCall& c, int B) {
  if (c.X.mode == PRO_BNBACK) {
    h->err = "internal: the block-sparse GEMM takes a stored dz (PRO_BNBACK is dW-only)";
    return LCN_E_ARG;
  }
  GemmArgs a{};
  a.X = c.X.p;
  a.S_in = c.X.S;
  a.blocks = c.blocks;
  a.ptr = c.ptr;
  a.idx = c.idx;
  a.order = c.order;
  a.tail = tail_groups();
  a.k_groups = c.k_groups;
  a.n_blocks = (c.ptr == h->fwd_ptr || c.ptr == h->bwd_ptr) ? h->nblk : h->nslab;  // hidden / thin layer
  a.bias = c.bias;
  a.pro_mode = c.X.mode;
  if (c.X.mode == PRO_BNACT) {
    a.pro_scale = h->bn[c.X.layer].scale;
    a.pro_shift = h->bn[c.X.layer].shift;
  }
  a.pro_F = h->F;
  a.spj_in = h->spj;
  a.alpha = h->alpha;
  a.Y = c.Y;
  a.S_out = c.S_out;
  a.addsrc = c.addsrc;
  a.epi_mode = c.epi_mode;
  a.stat = c.epi_mode != EPI_NONE ? h->stat_part : nullptr;
  if (c.epi_mode == EPI_BNBACK) {
    const BnStats& st = h->bn[c.epi_layer];
    a.epi_z = h->Z[c.epi_layer];
    a.epi_scale = st.scale;
    a.epi_shift = st.shift;
    a.epi_mean = st.mean;
    a.epi_rstd = st.rstd;
    a.epi_drop = drop_of(h, c.epi_layer, B);
  }
  a.epi_F = h->F;
  a.B = B;
  a.n_out_slabs = c.n_out_slabs;
  a.n_rt = (int)cdiv(B, kRT);
  // few row tiles: the kernel that splits the slab lists over a workgroup's
  // waves (no dropout epilogue there); its BN partials are per 32-row tile
  const bool small = a.n_rt <= h->small_rt && !(c.epi_mode == EPI_BNBACK && a.epi_drop.rate > 0.f);
  h->stat_rows = small ? kRT : kGemmRows;
  hipEvent_t ev[2];
  if (c.timer >= 0) tstart(h, c.timer, ev);
  if (!small && c.pair && c.pair->n > 0) {
    a.pairs = c.pair->pairs;
    a.ment = c.pair->ment;
    a.pair_order = c.pair->order;
    a.n_pairs = c.pair->n;
  }
  if (small) launch_gemm_bs_small(a, h->stream);
  else if (a.pairs) launch_gemm_bs_pair(a, h->stream);
  else launch_gemm_bs(a, h->stream);
  if (c.timer >= 0) tstop(h, c.timer, ev, c.flops_per_row * B);
  return LCN_OK;
}

// hidden layer k: forward (kindt = LCN_K_GEMM_FWD) or backward-data (LCN_K_GEMM_DX)
int gemm_hidden(Handle* h, int k, int kindt, const Operand& X, float* Y, const float* addsrc,
                int epi_mode, int epi_layer, int B) {
  const WLayer& Lr = h->wl[k];
  const bool fwd = kindt == LCN_K_GEMM_FWD;
  GemmCall c{X, fwd ? Lr.blk_fwd : Lr.blk_bwd, fwd ? h->fwd_ptr : h->bwd_ptr,
             fwd ? h->fwd_idx : h->bwd_idx, h->nslab, fwd ? h->theta + h->b_off[k] : nullptr,
             Y, h->nslab, addsrc, epi_mode, epi_layer,
             kindt, 2.0 * 4096.0 * h->nblk,   // 2*64*64 FLOP per block per row
             fwd ? h->fwd_order : h->bwd_order};
  c.pair = fwd ? &h->fwd_pair : &h->bwd_pair;
  return gemm(h, c, B);
}

// the workgroup map of a launch (make_dw_wgmap), uploaded once per batch size
int dw_map(Handle* h, Handle::DwGroups* g, const DwPlan& plan, int64_t B, const Handle::DwMap** out) {
  for (const auto& e : g->maps)
    if (e.B == B && e.plan.item_rows == plan.item_rows && e.plan.stride == plan.stride &&
        e.plan.n_slots == plan.n_slots && e.plan.sub == plan.sub) { *out = &e; return LCN_OK; }
  if (h->capturing) { h->err = "internal: weight-gradient map missing during graph capture"; return LCN_E_STATE; }
  if (g->maps.size() >= 64) {  // many batch sizes on one handle: start over (the maps are small)
    HIPC(hipStreamSynchronize(h->stream));
    for (auto& e : g->maps) {
      hipFree(e.dev);
      h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)e.dev));
    }
    g->maps.clear();
  }
  const std::vector<int4> map = make_dw_wgmap(g->n, plan, B);
  int4* dev = nullptr;
  CHECK(upload(h, &dev, map));
  g->maps.push_back(Handle::DwMap{B, plan, dev, (int)map.size()});
  *out = &g->maps.back();
  return LCN_OK;
}
// every map a step at batch B launches with (before a graph capture)
int dw_maps_ready(Handle* h, int64_t B) {
  const Handle::DwMap* m = nullptr;
  CHECK(dw_map(h, &h->grp_hidden, dw_plan(h, h->grp_hidden, h->nblk, B), B, &m));
  CHECK(dw_map(h, &h->grp_lift, dw_plan(h, h->grp_lift, h->nslab, B), B, &m));
  CHECK(dw_map(h, &h->grp_out, dw_plan(h, h->grp_out, h->nslab, B), B, &m));
  return LCN_OK;
}

// dW_e of a layer from A (input activations, raw or BN-apply prologue) and D
// (raw, or dz rebuilt from (dh, z) by the BN backward prologue -- then also
// stored to dz_out when given): partial slabs per batch chunk, then a
// fixed-order reduce into the raw-gradient vector (rows / columns past the
// valid range are padding and are dropped)
// `timer`: LCN_K_GEMM_DW (FLOPs), LCN_K_OUT_DW (algorithmic bytes) or -1 (not timed)
int gemm_dw(Handle* h, const Operand& A, const Operand& D, const int2* blk, int nblk, float* dW,
            int ld, int rows_valid, int cols_valid, int B, int timer, float* dz_out = nullptr) {
  GemmDwArgs a{};
  a.A = A.p;
  a.S_a = A.S;
  a.D = D.p;
  a.S_d = D.S;
  if (A.mode == PRO_BNACT) {
    a.pro_scale = h->bn[A.layer].scale;
    a.pro_shift = h->bn[A.layer].shift;
  }
  if (D.mode == PRO_BNBACK) {
    a.d_bnback = 1;
    a.d_scale = h->bn[D.layer].scale;
    a.d_shift = h->bn[D.layer].shift;
    a.d_z = h->Z[D.layer];
    a.d_c123 = h->batch_norm ? h->c123 : h->ident_c123;
    a.d_F = h->F;
    a.dz_out = dz_out;
    a.d_drop = drop_of(h, D.layer, B);
  }
  a.spj_a = h->spj;
  a.spj_d = h->spj;
  a.alpha = h->alpha;
  a.blk = blk;
  a.nblk = nblk;
  Handle::DwGroups* g = blk == h->blk ? &h->grp_hidden : blk == h->lift_blk ? &h->grp_lift
                        : blk == h->out_blk ? &h->grp_out : nullptr;
  if (!g) { h->err = "internal: unknown block list"; return LCN_E_ARG; }
  a.groups = g->dev;
  a.ngroups = g->n;
  a.B = B;
  a.plan = dw_plan(h, *g, nblk, B);
  if ((size_t)dw_plan_slots(a.plan) * nblk * 4096 > h->dw_cap) {
    h->err = "internal: weight-gradient partials exceed their buffer";
    return LCN_E_STATE;
  }
  const Handle::DwMap* m = nullptr;
  CHECK(dw_map(h, g, a.plan, B, &m));
  a.wgmap = m->dev;
  a.n_wg = m->n;
  // the kernel addresses its operands with 32-bit byte offsets
  if ((uint64_t)tiled_floats(B, std::max(A.S, D.S)) * 4 >= (1ull << 32)) {
    h->err = "batch too large for the weight-gradient kernel (an operand of 4 GB or more)";
    return LCN_E_ARG;
  }
  a.part = h->dw_part;
  hipEvent_t ev[2];
  if (timer >= 0) tstart(h, timer, ev);
  if (g->quad) launch_gemm_dw4(a, h->stream);
  else launch_gemm_dw(a, h->stream);
  if (timer >= 0)
    tstop(h, timer, ev, timer == LCN_K_GEMM_DW ? 2.0 * 4096.0 * nblk * B : 4.0 * (h->H + 51) * (double)B);
  launch_dw_reduce(h->dw_part, dw_plan_slots(a.plan), nblk, blk, dW, ld, rows_valid, cols_valid, h->stream);
  return LCN_OK;
}

// BN + LeakyReLU backward of BN layer k from the EPI_BNBACK partials (sum du,
// sum du*zhat) the GEMM producing its incoming gradient wrote: the dz
// coefficients c123 (consumed by the PRO_BNBACK prologues), the BN parameter
// grads and the bias grad.  dz itself is never materialised.
int bn_back(Handle* h, int k, int B) {
  hipStream_t s = h->stream;
  const BnStats& st = h->bn[k];
  const int bn = h->batch_norm;
  const double rows = (double)B;
  const RowInfo* ri = rinfo(h);
  const float* gamma = bn ? h->theta + h->gamma_off[k] : nullptr;
  float* dgam = bn ? h->rg + h->gamma_off[k] : nullptr;
  float* dbet = bn ? h->rg + h->beta_off[k] : nullptr;
  float* db = h->rg + h->b_off[k];
  const TilePartials tp = tile_partials(h, B);
  const BnRider none{};
  const int n_tiles = (int)cdiv(B, h->stat_rows);
  if ((!h->phased && !multi(h)) || !bn) {
    if (!tp.part)
      launch_colreduce_bn_bwd(h->stat_part, n_tiles, h->stat_rows, B, h->colacc, h->bn_ticket, h->H, h->F, 0, bn,
                              rows, ri, (double)B, gamma, st.mean, st.rstd, h->acc1, dgam, dbet, h->c123,
                              h->zsum[k], db, none, s);
    else
      launch_bn_bwd_finalize(h->colacc, tp, h->H, h->F, 0, bn, rows, ri, (double)B, gamma, st.mean, st.rstd,
                             h->acc1, dgam, dbet, h->c123, h->zsum[k], db, none, s);
    return LCN_OK;
  }
  // several ranks: the first BN backward of a step also carries the loss sum
  BnRider rider{};
  if (h->loss_pending) {
    rider.kind = kRideLoss;
    rider.loss = h->loss_sum;
    h->loss_pending = false;
  }
  if (!tp.part)
    launch_colreduce_bn_bwd(h->stat_part, n_tiles, h->stat_rows, B, h->colacc, h->bn_ticket, h->H, h->F, 1, bn,
                            rows, ri, (double)B, gamma, st.mean, st.rstd, h->acc1, dgam, dbet, h->c123,
                            h->zsum[k], db, rider, s);
  else
    launch_bn_bwd_finalize(h->colacc, tp, h->H, h->F, 1, bn, rows, ri, (double)B, gamma, st.mean, st.rstd,
                           h->acc1, dgam, dbet, h->c123, h->zsum[k], db, rider, s);
  CHECK(allreduce(h, h->acc1, 2 * h->F + rider_slots(rider), ncclDouble));
  launch_bn_bwd_finalize(h->colacc, tp, h->H, h->F, 2, bn, rows, ri, (double)B, gamma, st.mean, st.rstd,
                         h->acc1, dgam, dbet, h->c123, h->zsum[k], db, rider, s);
  return LCN_OK;
}

// BN apply + LeakyReLU (+ residual, + dropout) of BN layer k into a block
// output, timed as LCN_K_BN_ACT with its algorithmic HBM bytes
void bn_act_timed(Handle* h, const float* z, const float* res, float* out, int k, int B) {
  hipEvent_t ev[2];
  tstart(h, LCN_K_BN_ACT, ev);
  launch_bn_act(z, res, out, h->bn[k].scale, h->bn[k].shift, h->F, h->alpha, B, h->nslab,
                drop_of(h, k, B), h->stream);
  tstop(h, LCN_K_BN_ACT, ev, (res ? 3.0 : 2.0) * 4.0 * (double)B * h->H);
}

int forward(Handle* h, int B, bool with_labels, bool train) {
  hipStream_t s = h->stream;
  const int S = h->nslab, nl = h->nl;
  // tf.nn.dropout runs in training steps only (predict feeds rate 0, :102)
  h->drop_on = train && h->drop_rate > 0.f;
  // the ranks' batch rows: with BatchNorm they ride on BN layer 0's all-reduce (bn_stats)
  if (!h->batch_norm) CHECK(exchange_rows(h, B));
  CHECK(prep_weights(h));
  const int epi = h->batch_norm ? EPI_BNFWD : EPI_NONE;
  // lift z0 = x . W1e + b1 (models_att.py:714-729): x padded to one 64-wide slab
  // the thin layers are HBM-bound: their timers accumulate algorithmic bytes
  // per row (input read + output written)
  const double lift_bytes = 4.0 * (kJ * h->inF + h->H), out_bytes = 4.0 * (h->H + 51);
  CHECK(gemm(h, GemmCall{raw(h->x, 1), h->wl[0].blk_fwd, h->thin_ptr, h->thin_idx, S,
                         h->theta + h->b_off[0], h->Z[0], S, nullptr, epi, -1, LCN_K_LIFT, lift_bytes,
                         nullptr, (int)cdiv(kJ * h->inF, 8)}, B));
  CHECK(bn_stats(h, 0, B));
  bn_act_timed(h, h->Z[0], nullptr, h->Hb[0], 0, B);
  // two_linear blocks (models_att.py:630-705)
  for (int l = 0; l < h->L; ++l) {
    const int k1 = 2 * l + 1, k2 = 2 * l + 2;
    CHECK(gemm_hidden(h, k1, LCN_K_GEMM_FWD, raw(h->Hb[l], S), h->Z[k1], nullptr, epi, -1, B));
    CHECK(bn_stats(h, k1, B));
    // g = dropout(leaky(BN(z1))): fused into the next GEMM's operand load, or
    // materialised when dropout is on (the mask is per element, not per slab)
    Operand g{h->Z[k1], S, PRO_BNACT, k1};
    if (h->drop_on) {
      launch_bn_act(h->Z[k1], nullptr, h->Gb[l], h->bn[k1].scale, h->bn[k1].shift, h->F, h->alpha, B, S,
                    drop_of(h, k1, B), s);
      g = raw(h->Gb[l], S);
    }
    CHECK(gemm_hidden(h, k2, LCN_K_GEMM_FWD, g, h->Z[k2], nullptr, epi, -1, B));
    CHECK(bn_stats(h, k2, B));
    bn_act_timed(h, h->Z[k2], h->residual ? h->Hb[l] : nullptr, h->Hb[l + 1], k2, B);
  }
  // output layer y = h_L . W4e + b4 into a 1-slab buffer (51 used), then the
  // output assembly, loss and d out (models_att.py:749-773, :356)
  CHECK(gemm(h, GemmCall{raw(h->Hb[h->L], S), h->wl[nl - 1].blk_fwd, h->out_ptr, h->out_idx, 1,
                         nullptr, h->yout, 1, nullptr, EPI_NONE, -1, LCN_K_OUT, out_bytes}, B));
  OutAsmArgs oa{};
  oa.y = h->yout;
  oa.b4 = h->theta + h->b_off[nl - 1];
  oa.x = h->x;
  oa.in_f = h->inF;
  oa.lab = with_labels ? h->lab : nullptr;
  oa.out = h->out;
  oa.dy = train ? h->dy : nullptr;
  oa.loss_part = with_labels ? h->loss_part : nullptr;
  // a training step: the output bias gradient db4 = sum_b dy comes out of the same pass
  const bool want_db = train && with_labels;
  oa.db_part = want_db ? h->db_part : nullptr;
  oa.rows = (double)B;
  oa.ri = rinfo(h);
  oa.B = B;
  const int ogrid = (int)std::min<int64_t>(h->loss_grid, cdiv(B, 4));
  launch_out_assemble(oa, ogrid, s);
  if (with_labels)
    launch_loss_finalize(h->loss_part, ogrid, h->loss_sum, oa.db_part, h->rg + h->b_off[nl - 1], s);
  return LCN_OK;
}

int backward(Handle* h, int B) {
  const int nl = h->nl, L = h->L;
  const int H = h->H, S = h->nslab;
  const WLayer& Lo = h->wl[nl - 1];
  // Every dX GEMM stores the incoming gradient dh of the BN layer below it and
  // its epilogue reduces that layer's (sum du, sum du*zhat); bn_back turns
  // them into c123; the layer's dW GEMM rebuilds dz = c1 du + c2 + c3 z while
  // staging its D operand and stores it (DZ) for the layer's dX GEMM.
  // output layer: dh_L = dy . W4e^T (dy padded to 64 columns), dW4e = h_L^T dy, db4 = sum dy
  const int top = nl - 2;  // BN layer under the output layer
  CHECK(gemm(h, GemmCall{raw(h->dy, 1), Lo.blk_bwd, h->thin_ptr, h->thin_idx, S, nullptr,
                         h->DH, S, nullptr, EPI_BNBACK, top, -1, 0.0}, B));
  CHECK(gemm_dw(h, raw(h->Hb[L], S), raw(h->dy, 1), h->out_blk, S, h->rg + Lo.w_off, 51,
                H, 51, B, LCN_K_OUT_DW));
  // (db4 = sum_b dy was reduced with the loss, by out_assemble / loss_finalize)

  for (int l = L - 1; l >= 0; --l) {
    const int k1 = 2 * l + 1, k2 = 2 * l + 2;
    const int below = l > 0 ? k1 - 1 : 0;  // BN layer under block l's input h_l
    // DH = dh_{l+1}: gradient of the block output
    CHECK(bn_back(h, k2, B));
    const Operand g = h->drop_on ? raw(h->Gb[l], S) : Operand{h->Z[k1], S, PRO_BNACT, k1};
    CHECK(gemm_dw(h, g, Operand{h->DH, S, PRO_BNBACK, k2},
                  h->blk, h->nblk, h->rg + h->wl[k2].w_off, H, H, H, B, LCN_K_GEMM_DW,
                  h->DZ));                                             // dW_k2 = g^T dz2; DZ = dz2
    CHECK(gemm_hidden(h, k2, LCN_K_GEMM_DX, raw(h->DZ, S), h->DG, nullptr, EPI_BNBACK, k1, B));
    CHECK(bn_back(h, k1, B));
    CHECK(gemm_dw(h, raw(h->Hb[l], S), Operand{h->DG, S, PRO_BNBACK, k1}, h->blk, h->nblk,
                  h->rg + h->wl[k1].w_off, H, H, H, B, LCN_K_GEMM_DW,
                  h->DZ));                                             // dW_k1 = h_l^T dz1; DZ = dz1
    CHECK(gemm_hidden(h, k1, LCN_K_GEMM_DX, raw(h->DZ, S), h->DH, h->residual ? h->DH : nullptr,
                      EPI_BNBACK, below, B));                          // dh_l (+ residual)
  }
  // lift: dz0, dW1e = x^T dz0 (x padded: rows >= 17*in_F dropped), db1
  CHECK(bn_back(h, 0, B));
  CHECK(gemm_dw(h, raw(h->x, 1), Operand{h->DH, S, PRO_BNBACK, 0}, h->lift_blk, S,
                h->rg + h->wl[0].w_off, H, kJ * h->inF, H, B, -1));
  return LCN_OK;
}

// the device side of the update: mask / clip backward, Adam (lr_t from lr_dev)
int finish_device(Handle* h, bool update, bool keep_grads) {
  hipStream_t s = h->stream;
  if (multi(h)) CHECK(allreduce(h, h->rg, (size_t)h->P, ncclFloat));
  launch_wdot(h->rg, h->theta, h->w_offs, h->w_kin, h->w_nout, h->nl, h->blocksum, s);
  launch_maskgrad(h->blocksum, h->nl, h->Md, h->Sd, h->Cd, h->learnable, h->denom, h->norm2,
                  h->max_norm, h->learnable ? h->rg + h->mask_off : nullptr, h->lcoef, s);
  launch_adam(h->theta, h->m, h->v, h->rg, keep_grads ? h->gout : nullptr, h->segs, h->seg_start,
              h->nseg, h->adam_blocks, h->Md, h->lcoef, h->reg, h->lr_dev, h->b1, h->b2, h->adam_eps,
              update ? 1 : 0, s);
  return LCN_OK;
}

int stage_inputs(Handle* h, const float* x, const float* lab, int64_t B, int flags) {
  if (B <= 0 || B > h->Bmax) {
    h->err = "batch " + std::to_string(B) + " outside [1, max_batch=" + std::to_string(h->Bmax) + "]";
    return LCN_E_ARG;
  }
  const hipMemcpyKind kind = (flags & LCN_IN_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  // x lands in the 1-slab row-tiled operand of the lift GEMM (zero padded);
  // host input is staged row-major first
  if (x) {
    const int cols = kJ * h->inF;
    const float* src = x;
    if (!(flags & LCN_IN_DEVICE)) {
      HIPC(hipMemcpyAsync(h->xin, x, (size_t)B * cols * 4, hipMemcpyHostToDevice, h->stream));
      src = h->xin;
    }
    launch_tile_in(src, cols, (int)B, h->x, h->stream);
  }
  if (lab) HIPC(hipMemcpyAsync(h->lab, lab, (size_t)B * 51 * 4, kind, h->stream));
  h->lastB = B;
  return LCN_OK;
}

int finish_launches(Handle* h) {
  HIPC(hipGetLastError());
  return LCN_OK;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int lcn_abi_version(void) { return LCN_ABI_VERSION; }

const char* lcn_last_error(void* handle) {
  if (!handle) return g_create_error.c_str();
  return ((Handle*)handle)->err.c_str();
}

int lcn_create(const lcn_config* c, int device, void** handle) {
  g_create_error.clear();
  if (!c || !handle || !c->mask_matrix) { g_create_error = "null argument"; return LCN_E_ARG; }
  if (c->abi_version != LCN_ABI_VERSION) { g_create_error = "abi version mismatch"; return LCN_E_ARG; }
  if (c->joints != kJ) { g_create_error = "joints must be 17 (models_att.py:512-513, params_help.py:12)"; return LCN_E_ARG; }
  if (c->f <= 0 || c->f % kSlab) { g_create_error = "F must be a positive multiple of 64"; return LCN_E_ARG; }
  // the BN finish kernels keep 17*F float64 pairs in one workgroup's LDS (160 KiB)
  if (c->f > 512) { g_create_error = "F must be <= 512"; return LCN_E_ARG; }
  if (c->in_f != 2 && c->in_f != 3) { g_create_error = "in_F must be 2 or 3"; return LCN_E_ARG; }
  if (c->num_layers < 0 || c->max_batch <= 0) { g_create_error = "bad num_layers / max_batch"; return LCN_E_ARG; }
  if (c->max_batch > (int64_t)INT32_MAX / (kJ * c->f)) { g_create_error = "max_batch too large"; return LCN_E_ARG; }
  Handle* h = new Handle();
  h->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    g_create_error = std::string("HIP init: ") + hipGetErrorString(e);
    delete h;
    return LCN_E_HIP;
  }
  int rc = build(h, c);
  if (rc == LCN_OK) {
    hipError_t e2 = hipDeviceSynchronize();
    if (e2 != hipSuccess) { h->err = hipGetErrorString(e2); rc = LCN_E_HIP; }
  }
  if (rc != LCN_OK) {
    g_create_error = h->err;
    lcn_destroy(h);
    return rc;
  }
  *handle = h;
  return LCN_OK;
}

int lcn_destroy(void* handle) {
  if (!handle) return LCN_OK;
  Handle* h = (Handle*)handle;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  if (h->comm) ncclCommDestroy(h->comm);
  for (auto& t : h->timers)
    for (auto e : t.ev) hipEventDestroy(e);
  for (auto& g : h->graphs) hipGraphExecDestroy(g.exec);
  for (void* p : h->allocs) hipFree(p);
  for (void* p : h->user_bufs) if (p) hipFree(p);
  for (auto& d : h->datasets) if (d.ptr) hipFree(d.ptr);
  if (h->pred) hipFree(h->pred);
  if (h->pred_out) hipFree(h->pred_out);
  if (h->batch_losses) hipFree(h->batch_losses);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return LCN_OK;
}

int64_t lcn_num_params(void* handle) { return handle ? ((Handle*)handle)->P : -1; }

int lcn_param_layout(void* handle, int32_t index, char* name, int32_t cap, int64_t* offset,
                     int64_t* rows, int64_t* cols) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  if (index < 0 || index >= (int)h->specs.size()) return (int)h->specs.size();
  const ParamSpec& p = h->specs[index];
  if (name && cap > 0) {
    std::strncpy(name, p.name.c_str(), cap - 1);
    name[cap - 1] = 0;
  }
  if (offset) *offset = p.off;
  if (rows) *rows = p.rows;
  if (cols) *cols = p.cols;
  return LCN_OK;
}

static int copy_flat(Handle* h, float* dst, const float* src, int64_t n, hipMemcpyKind kind) {
  if (n != h->P) { h->err = "expected " + std::to_string(h->P) + " values"; return LCN_E_ARG; }
  HIPC(hipSetDevice(h->device));
  HIPC(hipStreamSynchronize(h->stream));
  HIPC(hipMemcpy(dst, src, (size_t)n * 4, kind));
  return LCN_OK;
}

int lcn_set_params(void* handle, const float* flat, int64_t n) {
  Handle* h = (Handle*)handle;
  if (!h || !flat) return LCN_E_ARG;
  return copy_flat(h, h->theta, flat, n, hipMemcpyHostToDevice);
}

int lcn_get_params(void* handle, float* flat, int64_t n) {
  Handle* h = (Handle*)handle;
  if (!h || !flat) return LCN_E_ARG;
  return copy_flat(h, flat, h->theta, n, hipMemcpyDeviceToHost);
}

int lcn_get_grads(void* handle, float* flat, int64_t n) {
  Handle* h = (Handle*)handle;
  if (!h || !flat) return LCN_E_ARG;
  if (!h->grads_valid) { h->err = "no gradients kept (pass LCN_KEEP_GRADS to lcn_train_step)"; return LCN_E_STATE; }
  return copy_flat(h, flat, h->gout, n, hipMemcpyDeviceToHost);
}

int lcn_set_optimizer_state(void* handle, const float* m, const float* v, int64_t n,
                            int64_t global_step, float b1p, float b2p) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  if (m) CHECK(copy_flat(h, h->m, m, n, hipMemcpyHostToDevice));
  if (v) CHECK(copy_flat(h, h->v, v, n, hipMemcpyHostToDevice));
  h->global_step = global_step;
  h->b1p = b1p;
  h->b2p = b2p;
  return LCN_OK;
}

int lcn_get_optimizer_state(void* handle, float* m, float* v, int64_t n, int64_t* global_step,
                            float* b1p, float* b2p) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  if (m) CHECK(copy_flat(h, m, h->m, n, hipMemcpyDeviceToHost));
  if (v) CHECK(copy_flat(h, v, h->v, n, hipMemcpyDeviceToHost));
  if (global_step) *global_step = h->global_step;
  if (b1p) *b1p = h->b1p;
  if (b2p) *b2p = h->b2p;
  return LCN_OK;
}

static int copy_out(Handle* h, float* out, int64_t B, int flags) {
  if (!out) return LCN_OK;
  if (flags & LCN_OUT_DEVICE) {
    HIPC(hipMemcpyAsync(out, h->out, (size_t)B * 51 * 4, hipMemcpyDeviceToDevice, h->stream));
  } else {
    HIPC(hipMemcpyAsync(out, h->out, (size_t)B * 51 * 4, hipMemcpyDeviceToHost, h->stream));
    HIPC(hipStreamSynchronize(h->stream));
  }
  return LCN_OK;
}

int lcn_forward(void* handle, const float* x, float* out, int64_t B, int32_t flags) {
  Handle* h = (Handle*)handle;
  if (!h || !x) return LCN_E_ARG;
  HIPC(hipSetDevice(h->device));
  CHECK(stage_inputs(h, x, nullptr, B, flags));
  CHECK(forward(h, (int)B, false, false));
  CHECK(finish_launches(h));
  CHECK(copy_out(h, out, B, flags));
  if (!(flags & LCN_ASYNC)) HIPC(hipStreamSynchronize(h->stream));
  return LCN_OK;
}

// mse (base_model.loss, models_att.py:356) + reg * sum(l2_loss(W), l2_loss(b))
// when regularisation is on (:362-365); the norms are those of this step's
// parameters (computed before the update)
static int read_loss(Handle* h, int64_t B, float* loss) {
  if (!loss) return LCN_OK;
  double v = 0.0;
  RowInfo ri{(double)B, 0};
  std::vector<double> n2(2 * h->nl, 0.0);
  HIPC(hipMemcpyAsync(&v, h->loss_sum, sizeof(double), hipMemcpyDeviceToHost, h->stream));
  if (multi(h))  // the mean is over every rank's rows
    HIPC(hipMemcpyAsync(&ri, h->rowinfo, sizeof(ri), hipMemcpyDeviceToHost, h->stream));
  if (h->reg != 0.f)
    HIPC(hipMemcpyAsync(n2.data(), h->norm2, n2.size() * sizeof(double), hipMemcpyDeviceToHost,
                        h->stream));
  HIPC(hipStreamSynchronize(h->stream));
  double l = v / (ri.rows_global * 51.0);
  if (h->reg != 0.f) {
    double r = 0.0;
    for (double x : n2) r += x / 2.0;
    l += (double)h->reg * r;
  }
  *loss = (float)l;
  return LCN_OK;
}

int lcn_forward_loss(void* handle, const float* x, const float* labels, float* out, int64_t B,
                     int32_t flags, float* loss) {
  Handle* h = (Handle*)handle;
  if (!h || !x || !labels) return LCN_E_ARG;
  HIPC(hipSetDevice(h->device));
  CHECK(stage_inputs(h, x, labels, B, flags));
  CHECK(forward(h, (int)B, true, false));
  if (multi(h)) CHECK(allreduce(h, h->loss_sum, 1, ncclDouble));
  CHECK(finish_launches(h));
  CHECK(copy_out(h, out, B, flags));
  CHECK(read_loss(h, B, loss));
  if (!(flags & LCN_ASYNC)) HIPC(hipStreamSynchronize(h->stream));
  return LCN_OK;
}

// forward, loss, backward and update of one step, enqueued on the stream
static int enqueue_step(Handle* h, int64_t B, bool update, bool keep) {
  CHECK(forward(h, (int)B, true, true));
  // the loss sum over the ranks: with BatchNorm it rides on the first BN
  // backward's all-reduce (bn_back), else it takes an all-reduce of its own
  if (multi(h)) {
    if (h->batch_norm) h->loss_pending = true;
    else CHECK(allreduce(h, h->loss_sum, 1, ncclDouble));
  }
  CHECK(backward(h, (int)B));
  h->loss_pending = false;
  return finish_device(h, update, keep);
}

// the captured graph of enqueue_step for (B, update, keep), made on first use
static int step_graph(Handle* h, int64_t B, bool update, bool keep, hipGraphExec_t* out) {
  for (const auto& g : h->graphs)
    if (g.B == B && g.update == update && g.keep == keep) { *out = g.exec; return LCN_OK; }
  hipGraph_t graph = nullptr;
  CHECK(dw_maps_ready(h, B));
  HIPC(hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed));
  h->capturing = true;
  const int rc = enqueue_step(h, B, update, keep);
  h->capturing = false;
  const hipError_t ec = hipStreamEndCapture(h->stream, &graph);
  if (rc != LCN_OK) { if (graph) hipGraphDestroy(graph); return rc; }
  if (ec != hipSuccess) { h->err = std::string("step graph capture: ") + hipGetErrorString(ec); return LCN_E_HIP; }
  hipGraphExec_t exec = nullptr;
  const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  hipGraphDestroy(graph);
  if (ei != hipSuccess) { h->err = std::string("step graph instantiate: ") + hipGetErrorString(ei); return LCN_E_HIP; }
  h->graphs.push_back(Handle::StepGraph{B, update, keep, exec});
  *out = exec;
  return LCN_OK;
}

static int run_train_step(Handle* h, int64_t B, int32_t flags, float* loss_out, float* lr_out) {
  const float lr = h->lr0 * powf(h->decay_rate, (float)h->global_step / (float)h->decay_steps);
  const float lr_t = lr * sqrtf(1.f - h->b2p) / (1.f - h->b1p);
  const bool update = !(flags & LCN_NO_UPDATE), keep = (flags & LCN_KEEP_GRADS) != 0;
  // dropout masks of this step: seed of training step number drop_calls
  h->step_seed = fmix32(h->drop_seed + fmix32((uint32_t)h->drop_calls + 0x9e3779b9u));
  if (h->drop_rate > 0.f) h->drop_calls++;
  uint32_t lr_bits;
  std::memcpy(&lr_bits, &lr_t, 4);
  HIPC(hipMemsetD32Async((hipDeviceptr_t)h->lr_dev, (int)lr_bits, 1, h->stream));
  hipGraphExec_t exec = nullptr;
  if (h->use_graphs && !multi(h) && !h->timing && h->drop_rate == 0.f &&
      step_graph(h, B, update, keep, &exec) != LCN_OK) {
    // capture unavailable: fall back to direct launches for this handle
    std::fprintf(stderr, "liblcn: step graph disabled (%s)\n", h->err.c_str());
    (void)hipGetLastError();
    h->err.clear();
    h->use_graphs = 0;
    exec = nullptr;
  }
  if (exec) {
    HIPC(hipGraphLaunch(exec, h->stream));
  } else {
    CHECK(enqueue_step(h, B, update, keep));
  }
  if (keep) h->grads_valid = 1;
  if (update) {
    h->b1p *= h->b1;
    h->b2p *= h->b2;
    h->global_step += 1;
  }
  CHECK(finish_launches(h));
  if (lr_out) *lr_out = lr;
  CHECK(read_loss(h, B, loss_out));
  if (!(flags & LCN_ASYNC)) HIPC(hipStreamSynchronize(h->stream));
  return LCN_OK;
}

int lcn_train_step(void* handle, const float* x, const float* labels, int64_t B, int32_t flags,
                   float* loss_out, float* lr_out) {
  Handle* h = (Handle*)handle;
  if (!h || !x || !labels) return LCN_E_ARG;
  HIPC(hipSetDevice(h->device));
  CHECK(stage_inputs(h, x, labels, B, flags));
  return run_train_step(h, B, flags, loss_out, lr_out);
}

// ---------------------------------------------------------------------------
// device-resident datasets
// ---------------------------------------------------------------------------
static int dataset_of(Handle* h, int32_t slot, Handle::Dataset** d) {
  if (slot < 0 || slot >= (int)h->datasets.size() || !h->datasets[slot].ptr) {
    h->err = "dataset slot " + std::to_string(slot) + " is empty (lcn_dataset_upload)";
    return LCN_E_ARG;
  }
  *d = &h->datasets[slot];
  return LCN_OK;
}

static int check_augment(Handle* h, const lcn_augment* a, Augment* out) {
  std::memset(out, 0, sizeof(*out));
  out->n_copies = 1;
  if (!a) return LCN_OK;
  if (a->n_copies < 1 || a->n_copies > LCN_MAX_COPIES) {
    h->err = "augment n_copies must be in [1, " + std::to_string(LCN_MAX_COPIES) + "]";
    return LCN_E_ARG;
  }
  out->n_copies = a->n_copies;
  for (int c = 0; c < a->n_copies; ++c) {
    if (a->op[c] < LCN_AUG_NONE || a->op[c] > LCN_AUG_TRANSLATE) {
      h->err = "unknown augment op " + std::to_string(a->op[c]);
      return LCN_E_ARG;
    }
    out->op[c] = a->op[c];
    out->p0[c] = a->param0[c];
    out->p1[c] = a->param1[c];
  }
  return LCN_OK;
}

int lcn_dataset_upload(void* handle, int32_t slot, const void* data, int32_t dtype, int64_t rows,
                       int32_t cols) {
  Handle* h = (Handle*)handle;
  if (!h || !data || slot < 0 || slot >= LCN_MAX_DATASETS || rows <= 0 || cols <= 0 ||
      (dtype != LCN_DTYPE_F32 && dtype != LCN_DTYPE_F64))
    return LCN_E_ARG;
  if (rows > (int64_t)INT32_MAX) { h->err = "dataset rows must fit int32 indices"; return LCN_E_ARG; }
  HIPC(hipSetDevice(h->device));
  HIPC(hipStreamSynchronize(h->stream));
  if ((int)h->datasets.size() <= slot) h->datasets.resize(slot + 1);
  Handle::Dataset& d = h->datasets[slot];
  const size_t bytes = (size_t)rows * cols * (dtype == LCN_DTYPE_F64 ? 8 : 4);
  if (d.ptr) { hipFree(d.ptr); d = Handle::Dataset(); }
  if (hipMalloc(&d.ptr, bytes) != hipSuccess) {
    d.ptr = nullptr;
    h->err = "hipMalloc dataset (" + std::to_string(bytes) + " bytes)";
    return LCN_E_NOMEM;
  }
  HIPC(hipMemcpy(d.ptr, data, bytes, hipMemcpyHostToDevice));
  d.dtype = dtype;
  d.rows = rows;
  d.cols = cols;
  return LCN_OK;
}

int lcn_dataset_free(void* handle, int32_t slot) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  if (slot < 0 || slot >= (int)h->datasets.size() || !h->datasets[slot].ptr) return LCN_OK;
  HIPC(hipSetDevice(h->device));
  HIPC(hipStreamSynchronize(h->stream));
  hipFree(h->datasets[slot].ptr);
  h->datasets[slot] = Handle::Dataset();
  return LCN_OK;
}

// build the batch (x tiles, labels) from dataset rows on the device
static int gather_batch(Handle* h, Handle::Dataset* dx, Handle::Dataset* dl, const int* idx_dev,
                        int64_t base, const Augment& aug, int64_t B) {
  launch_gather_x(dx->ptr, dx->dtype, dx->rows, h->inF, idx_dev, base, aug, (int)B, h->x, h->stream);
  if (dl) launch_gather_rows(dl->ptr, dl->dtype, dl->rows, 51, idx_dev, base, (int)B, h->lab, h->stream);
  h->lastB = B;
  return LCN_OK;
}

int lcn_train_step_indexed(void* handle, int32_t x_slot, int32_t lab_slot, const int32_t* idx,
                           int64_t B, int32_t flags, float* loss_out, float* lr_out) {
  Handle* h = (Handle*)handle;
  if (!h || !idx) return LCN_E_ARG;
  HIPC(hipSetDevice(h->device));
  Handle::Dataset *dx = nullptr, *dl = nullptr;
  CHECK(dataset_of(h, x_slot, &dx));
  CHECK(dataset_of(h, lab_slot, &dl));
  if (dx->cols != kJ * h->inF || dl->cols != 51 || dl->rows != dx->rows) {
    h->err = "dataset shapes: x must be [N][17*in_F], labels [N][51]";
    return LCN_E_ARG;
  }
  if (B <= 0 || B > h->Bmax) { h->err = "batch outside [1, max_batch]"; return LCN_E_ARG; }
  const int* id = (const int*)idx;
  if (!(flags & LCN_IN_DEVICE)) {
    HIPC(hipMemcpyAsync(h->idx_dev, idx, (size_t)B * 4, hipMemcpyHostToDevice, h->stream));
    id = h->idx_dev;
  }
  Augment none;
  CHECK(check_augment(h, nullptr, &none));
  CHECK(gather_batch(h, dx, dl, id, 0, none, B));
  return run_train_step(h, B, flags, loss_out, lr_out);
}

int lcn_predict_dataset(void* handle, int32_t x_slot, int32_t lab_slot, int64_t batch_size,
                        const lcn_augment* aug, const lcn_augment* undo, double* out,
                        int64_t out_rows, float* batch_losses, int64_t losses_cap,
                        int64_t* n_batches) {
  Handle* h = (Handle*)handle;
  if (!h || !out) return LCN_E_ARG;
  HIPC(hipSetDevice(h->device));
  Handle::Dataset *dx = nullptr, *dl = nullptr;
  CHECK(dataset_of(h, x_slot, &dx));
  if (lab_slot >= 0) CHECK(dataset_of(h, lab_slot, &dl));
  if (dx->cols != kJ * h->inF) { h->err = "x dataset must be [N][17*in_F]"; return LCN_E_ARG; }
  if (batch_size <= 0 || batch_size > h->Bmax) { h->err = "batch_size outside [1, max_batch]"; return LCN_E_ARG; }
  Augment a, u;
  CHECK(check_augment(h, aug, &a));
  CHECK(check_augment(h, undo, &u));
  if (u.n_copies != a.n_copies) { h->err = "augment / undo copy counts differ"; return LCN_E_ARG; }
  if (dl && (a.n_copies != 1 || dl->cols != 51 || dl->rows != dx->rows)) {
    h->err = "labels need [N][51] and no augmentation";
    return LCN_E_ARG;
  }
  const int64_t N = dx->rows, total = N * a.n_copies;
  if (out_rows < N) {
    h->err = "out holds " + std::to_string(out_rows) + " rows, the dataset has " + std::to_string(N);
    return LCN_E_ARG;
  }
  int64_t nb = cdiv(total, batch_size);
  if (multi(h)) {  // every rank runs the same number of (SyncBN) batches
    double v = (double)nb;
    CHECK(lcn_comm_allreduce_host(h, &v, 1, 1));
    nb = (int64_t)v;
  }
  if (h->pred_rows < total) {
    HIPC(hipStreamSynchronize(h->stream));
    if (h->pred) hipFree(h->pred);
    if (h->pred_out) hipFree(h->pred_out);
    h->pred = nullptr;
    h->pred_out = nullptr;
    h->pred_rows = 0;
    if (hipMalloc(&h->pred, (size_t)total * 51 * 8) != hipSuccess ||
        hipMalloc(&h->pred_out, (size_t)total * 51 * 8) != hipSuccess) {
      h->err = "hipMalloc predictions";
      return LCN_E_NOMEM;
    }
    h->pred_rows = total;
  }
  if (batch_losses && dl && nb > losses_cap) {
    h->err = "batch_losses holds " + std::to_string(losses_cap) + " < " + std::to_string(nb) + " batches";
    return LCN_E_ARG;
  }
  if (h->loss_cap < nb) {
    HIPC(hipStreamSynchronize(h->stream));
    if (h->batch_losses) hipFree(h->batch_losses);
    h->batch_losses = nullptr;
    h->loss_cap = 0;
    if (hipMalloc(&h->batch_losses, (size_t)nb * 4) != hipSuccess) { h->err = "hipMalloc losses"; return LCN_E_NOMEM; }
    h->loss_cap = nb;
  }
  // models_att.py:88-121: fixed batches over the (virtually concatenated)
  // copies, zero-padded last batch, batch-statistics BN
  for (int64_t i = 0; i < nb; ++i) {
    const int64_t begin = i * batch_size;
    CHECK(gather_batch(h, dx, dl, nullptr, begin, a, batch_size));
    CHECK(forward(h, (int)batch_size, dl != nullptr, false));
    if (dl) {
      if (multi(h)) CHECK(allreduce(h, h->loss_sum, 1, ncclDouble));
      launch_batch_loss(h->loss_sum, (double)batch_size, rinfo(h), h->batch_losses, (int)i, h->stream);
    }
    const int64_t n = std::min<int64_t>(batch_size, total - begin);
    if (n > 0) launch_store_pred(h->out, n, h->pred + begin * 51, h->stream);
  }
  const double* res = h->pred;
  if (a.n_copies > 1) {  // data.undo (data.py:269-287)
    launch_tta_undo(h->pred, N, u, h->pred_out, h->stream);
    res = h->pred_out;
  }
  CHECK(finish_launches(h));
  HIPC(hipMemcpyAsync(out, res, (size_t)N * 51 * 8, hipMemcpyDeviceToHost, h->stream));
  if (batch_losses && dl && nb > 0)
    HIPC(hipMemcpyAsync(batch_losses, h->batch_losses, (size_t)nb * 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(hipStreamSynchronize(h->stream));
  if (n_batches) *n_batches = nb;
  return LCN_OK;
}

int lcn_synchronize(void* handle) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  HIPC(hipSetDevice(h->device));
  HIPC(hipStreamSynchronize(h->stream));
  return LCN_OK;
}

int lcn_device_buffer(void* handle, int32_t slot, int64_t bytes, void** dptr) {
  Handle* h = (Handle*)handle;
  if (!h || slot < 0 || slot > 64 || bytes <= 0 || !dptr) return LCN_E_ARG;
  HIPC(hipSetDevice(h->device));
  if ((int)h->user_bufs.size() <= slot) {
    h->user_bufs.resize(slot + 1, nullptr);
    h->user_bytes.resize(slot + 1, 0);
  }
  if (h->user_bufs[slot] && h->user_bytes[slot] >= bytes) {
    *dptr = h->user_bufs[slot];
    return LCN_OK;
  }
  if (h->user_bufs[slot]) {
    HIPC(hipStreamSynchronize(h->stream));
    hipFree(h->user_bufs[slot]);
    h->user_bufs[slot] = nullptr;
  }
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) { h->err = "hipMalloc user buffer"; return LCN_E_NOMEM; }
  h->user_bufs[slot] = p;
  h->user_bytes[slot] = bytes;
  *dptr = p;
  return LCN_OK;
}

int lcn_memcpy_h2d(void* handle, void* dst, const void* src, int64_t bytes) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  HIPC(hipSetDevice(h->device));
  HIPC(hipStreamSynchronize(h->stream));
  HIPC(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return LCN_OK;
}

int lcn_memcpy_d2h(void* handle, void* dst, const void* src, int64_t bytes) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  HIPC(hipSetDevice(h->device));
  HIPC(hipStreamSynchronize(h->stream));
  HIPC(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return LCN_OK;
}

int lcn_comm_unique_id(void* id_out) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) { g_create_error = ncclGetErrorString(r); return LCN_E_COMM; }
  std::memcpy(id_out, &id, sizeof(id) < 128 ? sizeof(id) : 128);
  return LCN_OK;
}

int lcn_comm_init(void* handle, const void* id_in, int32_t rank, int32_t world) {
  Handle* h = (Handle*)handle;
  if (!h || !id_in || world < 1 || rank < 0 || rank >= world) return LCN_E_ARG;
  if (has_comm(h)) { h->err = "lcn_comm_init: the handle already has a communicator"; return LCN_E_ARG; }
  HIPC(hipSetDevice(h->device));
  CHECK(dalloc(h, &h->rows_all, (size_t)world));
  CHECK(dalloc(h, &h->acc1, (size_t)2 * h->F + world + 1));  // + the riders of the SyncBN all-reduces
  // a real communicator even at world 1: every exchange below is gated on
  // h->comm, so a one-GPU run after comm_init takes the multi-GPU code path
  // (phased BN reductions, RCCL all-reduces) end to end
  ncclUniqueId id;
  std::memcpy(&id, id_in, sizeof(id));
  NCCLC(ncclCommInitRank(&h->comm, world, id, rank));
  h->rank = rank;
  h->world = world;
  return LCN_OK;
}

int lcn_comm_init_host(void* handle, int32_t rank, int32_t world, lcn_host_allreduce_fn fn, void* ctx) {
  Handle* h = (Handle*)handle;
  if (!h || !fn || world < 1 || rank < 0 || rank >= world) return LCN_E_ARG;
  if (has_comm(h)) { h->err = "lcn_comm_init_host: the handle already has a communicator"; return LCN_E_ARG; }
  HIPC(hipSetDevice(h->device));
  CHECK(dalloc(h, &h->rows_all, (size_t)world));
  CHECK(dalloc(h, &h->acc1, (size_t)2 * h->F + world + 1));  // + the riders of the SyncBN all-reduces
  h->host_ar = fn;
  h->host_ctx = ctx;
  h->rank = rank;
  h->world = world;
  return LCN_OK;
}

int lcn_comm_suspend(void* handle, int32_t suspend) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  HIPC(hipSetDevice(h->device));
  HIPC(hipStreamSynchronize(h->stream));
  h->comm_off = suspend != 0;
  return LCN_OK;
}

int lcn_comm_allreduce_host(void* handle, double* values, int32_t count, int32_t op) {
  Handle* h = (Handle*)handle;
  if (!h || !values || count <= 0 || count > 2 * h->F) return LCN_E_ARG;
  if (!has_comm(h)) return LCN_OK;
  HIPC(hipSetDevice(h->device));
  HIPC(hipStreamSynchronize(h->stream));
  if (h->host_ar) {  // host values: no device round trip
    if (h->host_ar(h->host_ctx, values, count, LCN_DTYPE_F64, op == 1 ? 1 : 0) != 0) {
      h->err = "host all-reduce callback failed";
      return LCN_E_COMM;
    }
    return LCN_OK;
  }
  HIPC(hipMemcpy(h->acc2, values, count * sizeof(double), hipMemcpyHostToDevice));
  NCCLC(ncclAllReduce(h->acc2, h->acc2, count, ncclDouble, op == 1 ? ncclMax : ncclSum, h->comm,
                      h->stream));
  HIPC(hipStreamSynchronize(h->stream));
  HIPC(hipMemcpy(values, h->acc2, count * sizeof(double), hipMemcpyDeviceToHost));
  return LCN_OK;
}

int lcn_comm_info(void* handle, int32_t* kind, int32_t* rank, int32_t* world) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  int k = LCN_COMM_NONE, r = 0, w = 1;
  if (h->comm) {
    k = LCN_COMM_RCCL;
    NCCLC(ncclCommUserRank(h->comm, &r));
    NCCLC(ncclCommCount(h->comm, &w));
  } else if (h->host_ar) {
    k = LCN_COMM_HOST;
    r = h->rank;
    w = h->world;
  }
  if (kind) *kind = k;
  if (rank) *rank = r;
  if (world) *world = w;
  return LCN_OK;
}

int lcn_set_timing(void* handle, int32_t enable) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  HIPC(hipStreamSynchronize(h->stream));
  for (auto& t : h->timers) {
    for (auto e : t.ev) hipEventDestroy(e);
    t = Timer();
  }
  h->timer_err.clear();
  h->timing = enable;
  return LCN_OK;
}

int lcn_kernel_timing(void* handle, int32_t k, int64_t* launches, double* total_ms, double* flops) {
  Handle* h = (Handle*)handle;
  if (!h || k < 0 || k >= LCN_K_NUM) return LCN_E_ARG;
  HIPC(hipStreamSynchronize(h->stream));
  if (!h->timer_err.empty()) { h->err = h->timer_err; return LCN_E_HIP; }
  Timer& t = h->timers[k];
  double ms = 0.0;
  for (size_t i = 0; i + 1 < t.ev.size(); i += 2) {
    float e = 0.f;
    HIPC(hipEventElapsedTime(&e, t.ev[i], t.ev[i + 1]));
    ms += e;
  }
  if (launches) *launches = t.launches;
  if (total_ms) *total_ms = ms;
  if (flops) *flops = t.flops;
  return LCN_OK;
}

int lcn_debug_tensor(void* handle, int32_t kind, int32_t idx, float* host, int64_t n) {
  Handle* h = (Handle*)handle;
  if (!h || !host) return LCN_E_ARG;
  HIPC(hipStreamSynchronize(h->stream));
  const int64_t BH = h->lastB * h->H;
  const float* src = nullptr;
  int64_t cnt = 0;
  if (kind == 0 && idx >= 0 && idx < (int)h->Z.size()) { src = h->Z[idx]; cnt = BH; }
  else if (kind == 1 && idx >= 0 && idx < (int)h->Hb.size()) { src = h->Hb[idx]; cnt = BH; }
  else if (kind == 2 && idx >= 0 && idx < h->nbn) {
    if (n < 2 * h->F) return LCN_E_ARG;
    HIPC(hipMemcpy(host, h->bn[idx].mean, h->F * 4, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(host + h->F, h->bn[idx].rstd, h->F * 4, hipMemcpyDeviceToHost));
    return LCN_OK;
  } else if (kind == 3) { src = h->out; cnt = h->lastB * 51; }
  else if (kind == 5) {  // the lift operand x (1-slab row tiles) -> row-major [B][17*in_F]
    const int cols = kJ * h->inF;
    if (n < h->lastB * cols) { h->err = "buffer too small"; return LCN_E_ARG; }
    std::vector<float> t((size_t)tiled_floats(h->lastB, 1));
    HIPC(hipMemcpy(t.data(), h->x, t.size() * 4, hipMemcpyDeviceToHost));
    for (int64_t b = 0; b < h->lastB; ++b)
      for (int c = 0; c < cols; ++c) host[b * cols + c] = t[tix(b, c, 1)];
    return LCN_OK;
  } else if (kind == 6) { src = h->lab; cnt = h->lastB * 51; }
  else if (kind == 4) { src = h->rg; cnt = h->P; }
  else return LCN_E_ARG;
  if (n < cnt) { h->err = "buffer too small"; return LCN_E_ARG; }
  if (kind <= 1) {  // row-tiled activation -> row-major [B][H]
    const int S = h->nslab;
    std::vector<float> t((size_t)tiled_floats(h->lastB, S));
    HIPC(hipMemcpy(t.data(), src, t.size() * 4, hipMemcpyDeviceToHost));
    for (int64_t b = 0; b < h->lastB; ++b)
      for (int c = 0; c < h->H; ++c) host[b * h->H + c] = t[tix(b, c, S)];
    return LCN_OK;
  }
  HIPC(hipMemcpy(host, src, cnt * 4, hipMemcpyDeviceToHost));
  return LCN_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// evaluate.py's per-frame error loop (evaluate.py:53-73) as one launch:
// image_to_camera_frame (tools.py:183-194), optional Procrustes alignment
// (tools.py:96-202), per-joint Euclidean error.  Handle-free: it needs no
// network; errors are reported through lcn_last_error(NULL).
extern "C" int lcn_eval_mpjpe(int32_t device, int64_t n, const double* pred, const double* gt,
                              const double* box, const double* cam, const double* root_depth,
                              int32_t protocol2, double* err) {
  g_create_error.clear();
  if (n < 0 || (n > 0 && (!pred || !gt || !box || !cam || !root_depth || !err))) {
    g_create_error = "lcn_eval_mpjpe: null argument or negative frame count";
    return LCN_E_ARG;
  }
  if (n == 0) return LCN_OK;
  struct Guard {
    hipStream_t s = nullptr;
    double* d[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    ~Guard() {
      if (s) hipStreamSynchronize(s);
      for (double* p : d)
        if (p) hipFree(p);
      if (s) hipStreamDestroy(s);
    }
  } g;
  auto fail = [](const char* what, hipError_t e) {
    g_create_error = std::string("lcn_eval_mpjpe: ") + what + ": " + hipGetErrorString(e);
    return LCN_E_HIP;
  };
  hipError_t e;
  if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
  if ((e = hipStreamCreateWithFlags(&g.s, hipStreamNonBlocking)) != hipSuccess) return fail("stream", e);
  const size_t sz[6] = {(size_t)n * 51, (size_t)n * 51, (size_t)n * 4, (size_t)n * 4, (size_t)n,
                        (size_t)n * kJ};
  const double* src[5] = {pred, gt, box, cam, root_depth};
  for (int i = 0; i < 6; ++i) {
    if (hipMalloc(&g.d[i], sz[i] * sizeof(double)) != hipSuccess) {
      g.d[i] = nullptr;
      g_create_error = "lcn_eval_mpjpe: hipMalloc (" + std::to_string(sz[i] * 8) + " bytes)";
      return LCN_E_NOMEM;
    }
    if (i < 5 && (e = hipMemcpyAsync(g.d[i], src[i], sz[i] * sizeof(double), hipMemcpyHostToDevice, g.s)) !=
                     hipSuccess)
      return fail("copy in", e);
  }
  launch_mpjpe(n, g.d[0], g.d[1], g.d[2], g.d[3], g.d[4], protocol2 ? 1 : 0, g.d[5], g.s);
  if ((e = hipGetLastError()) != hipSuccess) return fail("launch", e);
  if ((e = hipMemcpyAsync(err, g.d[5], sz[5] * sizeof(double), hipMemcpyDeviceToHost, g.s)) != hipSuccess)
    return fail("copy out", e);
  if ((e = hipStreamSynchronize(g.s)) != hipSuccess) return fail("synchronize", e);
  return LCN_OK;
}

// tf.nn.dropout(rate) after every BN + LeakyReLU of the training step
// (models_att.py:673, 700, 742); masks from (seed, training-step counter),
// see lcn_internal.h Dropout.  rate 0 switches it off.
extern "C" int lcn_set_dropout(void* handle, float rate, uint64_t seed) {
  Handle* h = (Handle*)handle;
  if (!h) return LCN_E_ARG;
  if (!(rate >= 0.f && rate < 1.f)) { h->err = "dropout rate must be in [0, 1)"; return LCN_E_ARG; }
  HIPC(hipSetDevice(h->device));
  HIPC(hipStreamSynchronize(h->stream));
  if (rate > 0.f && h->Gb.empty()) {
    h->Gb.assign(h->L, nullptr);
    for (auto& g : h->Gb) CHECK(dalloc(h, &g, (size_t)tiled_floats(h->Bmax, h->nslab)));
  }
  h->drop_rate = rate;
  h->drop_scale = 1.f / (1.f - rate);  // TF: scale = 1 / (1 - rate) in float32
  h->drop_seed = (uint32_t)seed ^ (uint32_t)(seed >> 32);
  h->drop_calls = 0;
  return LCN_OK;
}
