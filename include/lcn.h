/*
 * lcn.h -- C ABI of liblcn.so, the MI355X-native locally-connected network
 * (LCN) hot path of adgx/lcn-pose.
 *
 * The reference's hot path is the TensorFlow graph built by
 * network/models_att.py (cgcnn._inference_lcn :707-775, base_model.loss
 * :352-380, base_model.training :382-421) and driven by one
 * tf.compat.v1.Session.run per step (fit :210-212, predict :112-121).  This
 * library replaces that graph + Session: every op of the forward, backward
 * and Adam update runs in hand-written HIP kernels for gfx950.  The Python
 * class network.models_att.cgcnn (lcn-pose_amd/network/models_att.py) keeps
 * the reference's API and calls these entry points through ctypes.
 *
 * Conventions
 *   - every function returns 0 on success, a negative LCN_E* code on error;
 *     lcn_last_error(h) (or lcn_last_error(NULL) for lcn_create failures)
 *     returns a message;
 *   - host buffers are C-contiguous float32 owned by the caller; device
 *     buffers are owned by the handle; one HIP stream per handle; a handle
 *     is not thread-safe (one handle per GPU, one process per GPU);
 *   - layouts are the reference's: input x[b, in_F*j + c], labels and
 *     output [b, 3*j + c]; flat parameters in TF variable-creation order
 *     (mask, w1, b1, bn gamma/beta, per block w2,b2,bn1,w3,b3,bn2, w4, b4),
 *     each tensor row-major as in the reference (W[i*Fin+p, j*Fout+q]).
 */
#ifndef LCN_H
#define LCN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LCN_ABI_VERSION 2

enum {
  LCN_OK = 0,
  LCN_E_ARG = -1,      /* bad argument / shape                       */
  LCN_E_HIP = -2,      /* HIP runtime error                          */
  LCN_E_NOMEM = -3,    /* device allocation failed                   */
  LCN_E_COMM = -4,     /* RCCL error                                 */
  LCN_E_STATE = -5     /* call not valid in the current state        */
};

/* mask kinds: cgcnn._initialize_mask (models_att.py:547-574) */
enum { LCN_MASK_LOCALLY_CONNECTED = 0, LCN_MASK_EXPONENTIAL = 1 };

/* flags for lcn_forward / lcn_train_step */
enum {
  LCN_IN_DEVICE = 1,      /* x / labels are device pointers (e.g. lcn_device_buffer) */
  LCN_OUT_DEVICE = 2,     /* out is a device pointer                                  */
  LCN_NO_UPDATE = 4,      /* train_step: compute gradients, skip the Adam update      */
  LCN_KEEP_GRADS = 8,     /* train_step: keep final dense gradients (lcn_get_grads)   */
  LCN_ASYNC = 16          /* do not synchronise the stream before returning           */
};

typedef struct lcn_config {
  int32_t abi_version;     /* = LCN_ABI_VERSION                                  */
  int32_t joints;          /* in_joints == out_joints == 17 (models_att.py:512-513) */
  int32_t in_f;            /* in_F, 2 or 3                                       */
  int32_t f;               /* F channels per joint, multiple of 64               */
  int32_t num_layers;      /* two_linear blocks                                  */
  int32_t mask_type;       /* LCN_MASK_*                                         */
  int32_t residual;        /* models_att.py:704                                  */
  int32_t batch_norm;      /* models_att.py:664, 693, 732                        */
  int32_t max_norm;        /* clip_by_norm(w, 1), models_att.py:659, 690, 726, 762 */
  int32_t reserved0;
  float bn_eps;            /* Keras BN epsilon, 1e-3                             */
  float leaky_alpha;       /* tf.nn.leaky_relu alpha, 0.2                        */
  float regularization;    /* 0 = off (models_att.py:362)                        */
  float learning_rate;     /* exponential_decay (models_att.py:392-399)          */
  float decay_rate;
  float beta1, beta2, adam_eps;
  int64_t decay_steps;
  int64_t max_batch;       /* largest per-call batch on this GPU                 */
  /* joints x joints, row = input joint i, column = output joint j:
   *   LC:  structure C[i][j] = (N^T)[i][j] != 0 (models_att.py:549, 571)
   *   EXP: the constant mask 2^-d (models_att.py:61, 574)                      */
  const float* mask_matrix;
} lcn_config;

/* --- lifetime --------------------------------------------------------- */
int lcn_create(const lcn_config* cfg, int device, void** handle);
int lcn_destroy(void* handle);
const char* lcn_last_error(void* handle);
int lcn_abi_version(void);

/* --- parameters / optimiser state (checkpoint I/O) ------------------- */
int64_t lcn_num_params(void* handle);
int lcn_param_layout(void* handle, int32_t index, char* name, int32_t name_cap,
                     int64_t* offset, int64_t* rows, int64_t* cols);
int lcn_set_params(void* handle, const float* flat, int64_t n);
int lcn_get_params(void* handle, float* flat, int64_t n);
int lcn_set_optimizer_state(void* handle, const float* m, const float* v, int64_t n,
                            int64_t global_step, float beta1_power, float beta2_power);
int lcn_get_optimizer_state(void* handle, float* m, float* v, int64_t n,
                            int64_t* global_step, float* beta1_power, float* beta2_power);
int lcn_get_grads(void* handle, float* flat, int64_t n);

/* --- compute ----------------------------------------------------------- */
/* predict one batch (models_att.py:79-132 inner body): out[B, 3*joints] */
int lcn_forward(void* handle, const float* x, float* out, int64_t batch, int32_t flags);
/* forward + mean-squared loss (predict with labels, models_att.py:108-115) */
int lcn_forward_loss(void* handle, const float* x, const float* labels, float* out,
                     int64_t batch, int32_t flags, float* loss);
/* one op_train (models_att.py:382-421): forward, loss, backward, Adam.
 * loss_out / lr_out may be NULL (then nothing is copied back). */
int lcn_train_step(void* handle, const float* x, const float* labels, int64_t batch,
                   int32_t flags, float* loss_out, float* lr_out);
int lcn_synchronize(void* handle);
/* tf.nn.dropout(rate) after every BN + LeakyReLU in training steps
 * (models_att.py:673, 700, 742; predict runs without it, :102).  rate in
 * [0, 1), 0 = off.  The masks are a counter-based hash of (seed, training-step
 * number since this call, layer, global row, column) -- see lcn_internal.h
 * Dropout; TF's own random stream cannot be reproduced. */
int lcn_set_dropout(void* handle, float rate, uint64_t seed);

/* --- device-resident data (on-device datasets; no host copies per step) */
int lcn_device_buffer(void* handle, int32_t slot, int64_t bytes, void** dptr);
int lcn_memcpy_h2d(void* handle, void* dst, const void* src, int64_t bytes);
int lcn_memcpy_d2h(void* handle, void* dst, const void* src, int64_t bytes);

/* --- device-resident datasets ------------------------------------------- */
/* The reference feeds every step from host numpy arrays: fit() fancy-indexes
 * the float64 train arrays with a permutation deque (models_att.py:193-212),
 * predict() slices fixed zero-padded batches (:88-121), inference.py
 * concatenates augmented copies before predict and undoes them after it
 * (inference.py:70-110, tools/data.py:10-54, 205-322).  These entry points keep
 * the arrays in HBM (in the caller's dtype; float64 is cast to float32 on the
 * device exactly as a float32 feed would) and build every batch there. */
enum { LCN_DTYPE_F32 = 0, LCN_DTYPE_F64 = 1 };
enum { LCN_MAX_DATASETS = 16, LCN_MAX_COPIES = 8 };
/* augmentation op per copy of the virtually concatenated dataset */
enum {
  LCN_AUG_NONE = 0,       /* identity                                           */
  LCN_AUG_FLIP = 1,       /* flip_data (data.py:10-25) / unflip_data (:236-249) */
  LCN_AUG_ROTATE = 2,     /* rotate_data (data.py:289-322): param0 = cos, param1 = sin of the angle,
                             computed by the caller as numpy does (np.cos(np.radians(a)))        */
  LCN_AUG_TRANSLATE = 3   /* translation_data (data.py:27-54): param0 = +t; as undo
                             (untranslation_data :205-218, all three coordinates): param0 = t */
};
typedef struct lcn_augment {
  int32_t n_copies;               /* 1 + number of augmentations                */
  int32_t op[LCN_MAX_COPIES];     /* op of copy c (copy 0 is normally NONE)      */
  double param0[LCN_MAX_COPIES];
  double param1[LCN_MAX_COPIES];
} lcn_augment;
/* copy rows x cols (row-major, dtype LCN_DTYPE_*) into dataset `slot` on the device */
int lcn_dataset_upload(void* handle, int32_t slot, const void* data, int32_t dtype, int64_t rows,
                       int32_t cols);
int lcn_dataset_free(void* handle, int32_t slot);
/* fit's step (models_att.py:194-212) on rows idx[0..B) of datasets x_slot
 * ([N][17*in_F]) and lab_slot ([N][51]); idx is host memory, or device memory
 * with LCN_IN_DEVICE.  Same flags / outputs as lcn_train_step. */
int lcn_train_step_indexed(void* handle, int32_t x_slot, int32_t lab_slot, const int32_t* idx,
                           int64_t batch, int32_t flags, float* loss_out, float* lr_out);
/* predict (models_att.py:79-132) over the whole dataset x_slot, virtually
 * concatenated as aug->n_copies augmented copies (aug NULL = one plain copy):
 * fixed batches of batch_size, the last zero-padded, batch-statistics BN.
 * With more than one copy the predictions are undone per copy by `undo` and
 * averaged (data.undo).  out: host float64 [N][51], N = the dataset's rows;
 * out_rows is the capacity of `out` in rows (LCN_E_ARG if < N).  lab_slot >= 0 (no
 * augmentation): batch_losses[i] receives batch i's float32 mean loss
 * (losses_cap >= number of batches).  With world > 1 every rank predicts its
 * own shard and the ranks' batch i together form one SyncBN batch. */
int lcn_predict_dataset(void* handle, int32_t x_slot, int32_t lab_slot, int64_t batch_size,
                        const lcn_augment* aug, const lcn_augment* undo, double* out,
                        int64_t out_rows, float* batch_losses, int64_t losses_cap,
                        int64_t* n_batches);

/* --- data parallel (RCCL over xGMI) ------------------------------------ */
/* Replaces the single-process Session of models_att.py:155, 210-212 with one
 * process per GPU.  lcn_comm_init creates an RCCL communicator at any world
 * size (world 1 included: the multi-GPU path then runs on one GPU) and may be
 * called once per handle (LCN_E_ARG otherwise).  After it, every step does
 * SyncBN (phased BN reductions + ncclAllReduce, float64) and one float32
 * all-reduce of the raw gradient vector on the handle's stream: 4L + 3
 * collectives per training step with L blocks (the ranks' batch rows ride on
 * BN layer 0's all-reduce, the loss sum on the first BN backward's).
 * lcn_comm_allreduce_host: count <= 2F doubles, a no-op without a
 * communicator. */
int lcn_comm_unique_id(void* id_out /* 128 bytes */);
int lcn_comm_init(void* handle, const void* id /* 128 bytes */, int32_t rank, int32_t world);
/* The same data-parallel step over a transport of the caller's: every exchange
 * (the ranks' row counts, SyncBN sums, the loss, the raw gradient vector)
 * copies its device buffer to host memory, calls fn -- an in-place all-reduce
 * of `count` elements (dtype LCN_DTYPE_F32 / LCN_DTYPE_F64; op 0 sum, 1 max)
 * over the `world` ranks, 0 on success -- and copies the result back, in
 * stream order.  For ranks that RCCL cannot join (several ranks sharing one
 * GPU, as the multi-rank tests do; a host-only fabric).  The ranks' batches
 * may differ in size with either communicator: BN statistics, the loss and
 * its gradient use the all-reduced global row count.  No counterpart in the
 * reference (single process, models_att.py:155). */
typedef int (*lcn_host_allreduce_fn)(void* ctx, void* buf, int64_t count, int32_t dtype, int32_t op);
int lcn_comm_init_host(void* handle, int32_t rank, int32_t world, lcn_host_allreduce_fn fn, void* ctx);
/* suspend != 0: until resumed, compute calls on this handle run rank-locally
 * (no exchange, BN over the call's own batch) -- every rank can then evaluate
 * the same whole data set with the single-process arithmetic of predict
 * (models_att.py:79-132) between data-parallel training steps.  Every rank
 * must suspend / resume at the same point.  lcn_comm_allreduce_host still
 * exchanges while suspended. */
int lcn_comm_suspend(void* handle, int32_t suspend);
int lcn_comm_allreduce_host(void* handle, double* values, int32_t count, int32_t op /* 0 sum, 1 max */);
/* What joins this handle to other ranks: kind LCN_COMM_*; rank / world as the
 * communicator itself reports them (RCCL: ncclCommUserRank / ncclCommCount of
 * the live communicator, so a caller can show that RCCL holds `world` ranks),
 * 0 / 1 without one.  Any out pointer may be NULL.  No counterpart in the
 * reference (single process, models_att.py:155). */
enum { LCN_COMM_NONE = 0, LCN_COMM_RCCL = 1, LCN_COMM_HOST = 2 };
int lcn_comm_info(void* handle, int32_t* kind, int32_t* rank, int32_t* world);

/* --- evaluation --------------------------------------------------------- */
/* evaluate.py's per-frame loop (evaluate.py:53-73) in one launch, float64:
 * every frame's prediction goes from the image frame to the camera frame
 * (tools/tools.py:183-194: box width / 2000 depth ratio, root depth, pinhole
 * cx, cy, fx, fy), is Procrustes-aligned to the ground truth when protocol2
 * != 0 (align_to_gt = procrustes(gt, pred)[1], tools.py:96-202), and
 * err[f][j] = |pred_j - gt_j| (evaluate.py:61).
 *   pred [n][17][3] image-frame predictions (inference.py's result rows)
 *   gt   [n][17][3] joint_3d_camera        box [n][4] (x0, y0, x1, y1)
 *   cam  [n][4] (cx, cy, fx, fy)           root_depth [n]
 * Host arrays in, host err [n][17] out; no handle (errors: lcn_last_error(NULL)).
 * Protocol 1 is bit-identical to the reference's numpy; protocol 2 agrees to
 * rounding (a Jacobi SVD instead of LAPACK's). */
int lcn_eval_mpjpe(int32_t device, int64_t n, const double* pred, const double* gt, const double* box,
                   const double* cam, const double* root_depth, int32_t protocol2, double* err);

/* lcn_eval_mpjpe for callers that cannot allocate device memory (harnesses
 * that forbid hipMalloc, tight evaluation loops): same arguments, results
 * and errors, but the host arrays are staged in a fixed per-GPU array of the
 * library (LCN_EVAL_STATIC_MAX_FRAMES frames, 1 KiB each; every GPU the
 * library runs on holds it until the process ends) on the null stream, so the
 * call makes no hipMalloc / hipFree / stream creation.  n beyond the limit is
 * LCN_E_ARG.  Calls that overlap on one GPU race on that array: serialise
 * them.  Errors: lcn_last_error(NULL).  No counterpart in the reference. */
#define LCN_EVAL_STATIC_MAX_FRAMES 16384
int lcn_eval_mpjpe_static(int32_t device, int64_t n, const double* pred, const double* gt,
                          const double* box, const double* cam, const double* root_depth,
                          int32_t protocol2, double* err);

/* --- checkpoint I/O helpers (host only) -------------------------------- */
/* CRC-32C of TensorFlow tensor-bundle checkpoints (tf.train.Saver files the
 * reference writes and restores, models_att.py:256-260, 321-322, 457-461):
 * leveldb/TF crc32c::Extend -- `crc` is the unmasked CRC of the preceding
 * bytes (0 to start).  Used by lcn_amd/tf_bundle.py. */
uint32_t lcn_crc32c(uint32_t crc, const void* data, int64_t n);

/* --- instrumentation --------------------------------------------------- */
/* kernel ids for lcn_kernel_timing */
/* LCN_K_BN_ACT: the BN apply + LeakyReLU (+ residual) pass that materialises
 * the block outputs; LCN_K_LIFT / LCN_K_OUT / LCN_K_OUT_DW: the thin lift
 * (models_att.py:729) and output (:765) layers' forward launches and the
 * output layer's weight gradient.  For these HBM-bound kernels the "flops"
 * field accumulates algorithmic HBM bytes (inputs read + outputs written).
 * LCN_K_COMM: the all-reduces of a step on a joined handle (RCCL or the host
 * exchange), from enqueue to completion on the compute stream -- so with the
 * wait for the slowest rank; "flops" accumulates the bytes reduced. */
enum { LCN_K_GEMM_FWD = 0, LCN_K_GEMM_DX = 1, LCN_K_GEMM_DW = 2, LCN_K_BN_ACT = 3, LCN_K_LIFT = 4,
       LCN_K_OUT = 5, LCN_K_OUT_DW = 6, LCN_K_COMM = 7, LCN_K_NUM = 8 };
/* enable: 0 = off, 1 = HIP-event timers around every kernel class above, or a
 * set of bits 1 << (1 + LCN_K_x) to time only those classes (timing-only
 * events: two records per timed launch, no system fence).  Resets the accumulated timings. */
int lcn_set_timing(void* handle, int32_t enable);
int lcn_kernel_timing(void* handle, int32_t kernel, int64_t* launches, double* total_ms,
                      double* flops);
/* debug: copy an internal activation to host.  kind 0 = z (pre-BN) of linear
 * layer idx, 1 = block output h_idx, 2 = BN (mean, rstd) of BN layer idx,
 * 3 = output [B][51], 4 = raw gradient vector, 5 = the batch's input x
 * [B][17*in_F] as the lift layer sees it, 6 = the batch's labels [B][51] */
int lcn_debug_tensor(void* handle, int32_t kind, int32_t idx, float* host, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* LCN_H */
