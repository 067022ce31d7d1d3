"""ctypes binding of liblcn.so (the C ABI in include/lcn.h).

There is no fallback: if the HIP library is missing or fails to load, every
constructor raises ``LcnNativeError`` -- the product path never computes on
the CPU.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LCN_LIB", os.path.join(HERE, "liblcn.so"))

LCN_ABI_VERSION = 2
MASK_LOCALLY_CONNECTED, MASK_EXPONENTIAL = 0, 1
IN_DEVICE, OUT_DEVICE, NO_UPDATE, KEEP_GRADS, ASYNC = 1, 2, 4, 8, 16
K_GEMM_FWD, K_GEMM_DX, K_GEMM_DW, K_BN_ACT, K_LIFT, K_OUT, K_OUT_DW, K_COMM = 0, 1, 2, 3, 4, 5, 6, 7
DTYPE_F32, DTYPE_F64 = 0, 1
MAX_DATASETS, MAX_COPIES = 16, 8
AUG_NONE, AUG_FLIP, AUG_ROTATE, AUG_TRANSLATE = 0, 1, 2, 3

# every entry point include/lcn.h declares, with its ctypes signature
_i32, _i64, _f32p, _vp = ctypes.c_int32, ctypes.c_int64, ctypes.POINTER(ctypes.c_float), ctypes.c_void_p
_f64p, _i64p = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)


class LcnConfig(ctypes.Structure):
    _fields_ = [("abi_version", _i32), ("joints", _i32), ("in_f", _i32), ("f", _i32),
                ("num_layers", _i32), ("mask_type", _i32), ("residual", _i32),
                ("batch_norm", _i32), ("max_norm", _i32), ("reserved0", _i32),
                ("bn_eps", ctypes.c_float), ("leaky_alpha", ctypes.c_float),
                ("regularization", ctypes.c_float), ("learning_rate", ctypes.c_float),
                ("decay_rate", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("adam_eps", ctypes.c_float),
                ("decay_steps", _i64), ("max_batch", _i64), ("mask_matrix", _f32p)]


class LcnAugment(ctypes.Structure):
    _fields_ = [("n_copies", _i32), ("op", _i32 * MAX_COPIES),
                ("param0", ctypes.c_double * MAX_COPIES), ("param1", ctypes.c_double * MAX_COPIES)]


def make_augment(ops) -> LcnAugment:
    """ops: list of (op, param0, param1) per copy of the virtual dataset."""
    a = LcnAugment()
    if not 1 <= len(ops) <= MAX_COPIES:
        raise ValueError(f"1..{MAX_COPIES} copies supported, got {len(ops)}")
    a.n_copies = len(ops)
    for c, (op, p0, p1) in enumerate(ops):
        a.op[c], a.param0[c], a.param1[c] = int(op), float(p0), float(p1)
    return a


# lcn_host_allreduce_fn: int (*)(void* ctx, void* buf, int64 count, int32 dtype, int32 op)
HOST_ALLREDUCE_FN = ctypes.CFUNCTYPE(_i32, _vp, _vp, _i64, _i32, _i32)

SIGNATURES = {
    "lcn_abi_version": ([], _i32),
    "lcn_create": ([ctypes.POINTER(LcnConfig), _i32, ctypes.POINTER(_vp)], _i32),
    "lcn_destroy": ([_vp], _i32),
    "lcn_last_error": ([_vp], ctypes.c_char_p),
    "lcn_num_params": ([_vp], _i64),
    "lcn_param_layout": ([_vp, _i32, ctypes.c_char_p, _i32, _i64p, _i64p, _i64p], _i32),
    "lcn_set_params": ([_vp, _f32p, _i64], _i32),
    "lcn_get_params": ([_vp, _f32p, _i64], _i32),
    "lcn_set_optimizer_state": ([_vp, _f32p, _f32p, _i64, _i64, ctypes.c_float, ctypes.c_float], _i32),
    "lcn_get_optimizer_state": ([_vp, _f32p, _f32p, _i64, _i64p, _f32p, _f32p], _i32),
    "lcn_get_grads": ([_vp, _f32p, _i64], _i32),
    "lcn_forward": ([_vp, _vp, _vp, _i64, _i32], _i32),
    "lcn_forward_loss": ([_vp, _vp, _vp, _vp, _i64, _i32, _f32p], _i32),
    "lcn_train_step": ([_vp, _vp, _vp, _i64, _i32, _f32p, _f32p], _i32),
    "lcn_synchronize": ([_vp], _i32),
    "lcn_device_buffer": ([_vp, _i32, _i64, ctypes.POINTER(_vp)], _i32),
    "lcn_memcpy_h2d": ([_vp, _vp, _vp, _i64], _i32),
    "lcn_memcpy_d2h": ([_vp, _vp, _vp, _i64], _i32),
    "lcn_dataset_upload": ([_vp, _i32, _vp, _i32, _i64, _i32], _i32),
    "lcn_dataset_free": ([_vp, _i32], _i32),
    "lcn_train_step_indexed": ([_vp, _i32, _i32, _vp, _i64, _i32, _f32p, _f32p], _i32),
    "lcn_predict_dataset": ([_vp, _i32, _i32, _i64, ctypes.POINTER(LcnAugment),
                             ctypes.POINTER(LcnAugment), _f64p, _i64, _f32p, _i64, _i64p], _i32),
    "lcn_comm_unique_id": ([_vp], _i32),
    "lcn_comm_init": ([_vp, _vp, _i32, _i32], _i32),
    "lcn_comm_init_host": ([_vp, _i32, _i32, HOST_ALLREDUCE_FN, _vp], _i32),
    "lcn_comm_suspend": ([_vp, _i32], _i32),
    "lcn_comm_allreduce_host": ([_vp, _f64p, _i32, _i32], _i32),
    "lcn_comm_info": ([_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i32), ctypes.POINTER(_i32)], _i32),
    "lcn_crc32c": ([ctypes.c_uint32, ctypes.c_char_p, _i64], ctypes.c_uint32),
    "lcn_set_dropout": ([_vp, ctypes.c_float, ctypes.c_uint64], _i32),
    "lcn_eval_mpjpe": ([_i32, _i64, _f64p, _f64p, _f64p, _f64p, _f64p, _i32, _f64p], _i32),
    "lcn_eval_mpjpe_static": ([_i32, _i64, _f64p, _f64p, _f64p, _f64p, _f64p, _i32, _f64p], _i32),
    "lcn_set_timing": ([_vp, _i32], _i32),
    "lcn_kernel_timing": ([_vp, _i32, _i64p, _f64p, _f64p], _i32),
    "lcn_debug_tensor": ([_vp, _i32, _i32, _f32p, _i64], _i32),
}


class LcnNativeError(RuntimeError):
    pass


_LIB = None


def load_library(path: Optional[str] = None):
    """Load liblcn.so (raises LcnNativeError if it is missing)."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise LcnNativeError(f"liblcn.so not found at {p}: build it with "
                             f"`python -c 'import __graft_entry__ as g; g.build()'`")
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:
        raise LcnNativeError(f"cannot load {p}: {e}") from e
    for name, (args, res) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if lib.lcn_abi_version() != LCN_ABI_VERSION:
        raise LcnNativeError("liblcn.so ABI version mismatch")
    if path is None:
        _LIB = lib
    return lib


EVAL_STATIC_MAX_FRAMES = 16384


def eval_mpjpe(pred, gt, box, cam, root_depth, protocol2: bool = False, device: int = 0,
               static: bool = False) -> np.ndarray:
    """Per-frame, per-joint camera-space error of evaluate.py's loop
    (evaluate.py:53-73) in one device launch (lcn_eval_mpjpe).

    pred [N, 17, 3] image-frame predictions, gt [N, 17, 3] joint_3d_camera,
    box [N, 4], cam [N, 4] = (cx, cy, fx, fy), root_depth [N]; all float64.
    Returns err [N, 17] float64.  static=True: the allocation-free entry point
    (lcn_eval_mpjpe_static, at most EVAL_STATIC_MAX_FRAMES frames per call)."""
    lib = load_library()
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (pred, gt, box, cam, root_depth)]
    n = arrs[0].shape[0]
    shapes = [(n, 17, 3), (n, 17, 3), (n, 4), (n, 4), (n,)]
    for a, shp, name in zip(arrs, shapes, ("pred", "gt", "box", "cam", "root_depth")):
        if a.shape != shp:
            raise ValueError(f"{name} has shape {a.shape}, expected {shp}")
    err = np.empty((n, 17), np.float64)
    ptr = [a.ctypes.data_as(_f64p) for a in arrs]
    if static:
        rc = lib.lcn_eval_mpjpe_static(device, n, *ptr, 1 if protocol2 else 0, err.ctypes.data_as(_f64p))
        if rc != 0:
            raise LcnNativeError(f"lcn_eval_mpjpe_static failed ({rc}): "
                                 f"{lib.lcn_last_error(None).decode()}")
        return err
    rc = lib.lcn_eval_mpjpe(device, n, *ptr, 1 if protocol2 else 0, err.ctypes.data_as(_f64p))
    if rc != 0:
        raise LcnNativeError(f"lcn_eval_mpjpe failed ({rc}): {lib.lcn_last_error(None).decode()}")
    return err


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_f32p)


def _as_f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


class DeviceBuffer:
    """A device allocation owned by a Network handle (slot-addressed)."""

    def __init__(self, net: "Network", slot: int, nbytes: int):
        self.net, self.slot, self.nbytes = net, slot, nbytes
        p = _vp()
        net._check(net.lib.lcn_device_buffer(net.h, slot, nbytes, ctypes.byref(p)))
        self.ptr = p.value

    def upload(self, arr: np.ndarray, offset_bytes: int = 0):
        a = np.ascontiguousarray(arr)
        assert offset_bytes + a.nbytes <= self.nbytes
        self.net._check(self.net.lib.lcn_memcpy_h2d(self.net.h, self.ptr + offset_bytes,
                                                    a.ctypes.data, a.nbytes))

    def download(self, arr: np.ndarray, offset_bytes: int = 0):
        assert arr.flags["C_CONTIGUOUS"] and offset_bytes + arr.nbytes <= self.nbytes
        self.net._check(self.net.lib.lcn_memcpy_d2h(self.net.h, arr.ctypes.data,
                                                    self.ptr + offset_bytes, arr.nbytes))


class Network:
    """One LCN replica on one GPU (a liblcn handle)."""

    def __init__(self, *, F=64, in_F=2, num_layers=3, mask_type="locally_connected",
                 mask_matrix: np.ndarray, residual=True, batch_norm=True, max_norm=True,
                 regularization=0.0, learning_rate=1e-3, decay_steps=32000, decay_rate=0.96,
                 bn_eps=1e-3, leaky_alpha=0.2, beta1=0.9, beta2=0.999, adam_eps=1e-8,
                 max_batch=256, device=0):
        self.lib = load_library()
        self._mask = _as_f32(mask_matrix).reshape(17, 17).copy()
        cfg = LcnConfig()
        cfg.abi_version = LCN_ABI_VERSION
        cfg.joints, cfg.in_f, cfg.f, cfg.num_layers = 17, in_F, F, num_layers
        cfg.mask_type = MASK_LOCALLY_CONNECTED if "locally_connected" in mask_type else MASK_EXPONENTIAL
        cfg.residual, cfg.batch_norm, cfg.max_norm = int(residual), int(batch_norm), int(max_norm)
        cfg.bn_eps, cfg.leaky_alpha = bn_eps, leaky_alpha
        cfg.regularization = 0.0 if regularization in (None, 0) else float(regularization)
        cfg.learning_rate, cfg.decay_rate, cfg.decay_steps = learning_rate, decay_rate, decay_steps
        cfg.beta1, cfg.beta2, cfg.adam_eps = beta1, beta2, adam_eps
        cfg.max_batch = int(max_batch)
        cfg.mask_matrix = _fp(self._mask)
        self.cfg = cfg
        self.F, self.in_F, self.max_batch = F, in_F, int(max_batch)
        h = _vp()
        rc = self.lib.lcn_create(ctypes.byref(cfg), device, ctypes.byref(h))
        if rc != 0:
            raise LcnNativeError(f"lcn_create failed ({rc}): {self.lib.lcn_last_error(None).decode()}")
        self.h = h
        self.n_params = int(self.lib.lcn_num_params(self.h))

    # -- lifetime
    def close(self):
        if getattr(self, "h", None):
            self.lib.lcn_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise LcnNativeError(f"liblcn error {rc}: {self.lib.lcn_last_error(self.h).decode()}")

    # -- parameters
    def param_layout(self) -> List[Tuple[str, int, Tuple[int, ...]]]:
        out, i = [], 0
        name = ctypes.create_string_buffer(64)
        off, r, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        while self.lib.lcn_param_layout(self.h, i, name, 64, ctypes.byref(off), ctypes.byref(r),
                                        ctypes.byref(c)) == 0:
            shape = (c.value,) if r.value == 1 else (r.value, c.value)
            out.append((name.value.decode(), off.value, shape))
            i += 1
        return out

    def set_params(self, flat: np.ndarray):
        f = _as_f32(flat).ravel()
        self._check(self.lib.lcn_set_params(self.h, _fp(f), f.size))

    def get_params(self) -> np.ndarray:
        f = np.empty(self.n_params, np.float32)
        self._check(self.lib.lcn_get_params(self.h, _fp(f), f.size))
        return f

    def get_grads(self) -> np.ndarray:
        f = np.empty(self.n_params, np.float32)
        self._check(self.lib.lcn_get_grads(self.h, _fp(f), f.size))
        return f

    def set_optimizer_state(self, m, v, global_step, beta1_power, beta2_power):
        m = None if m is None else _as_f32(m).ravel()
        v = None if v is None else _as_f32(v).ravel()
        self._check(self.lib.lcn_set_optimizer_state(
            self.h, None if m is None else _fp(m), None if v is None else _fp(v), self.n_params,
            int(global_step), float(beta1_power), float(beta2_power)))

    def get_optimizer_state(self):
        m = np.empty(self.n_params, np.float32)
        v = np.empty(self.n_params, np.float32)
        gs, b1p, b2p = ctypes.c_int64(), ctypes.c_float(), ctypes.c_float()
        self._check(self.lib.lcn_get_optimizer_state(self.h, _fp(m), _fp(v), self.n_params,
                                                     ctypes.byref(gs), ctypes.byref(b1p),
                                                     ctypes.byref(b2p)))
        return m, v, gs.value, b1p.value, b2p.value

    # -- compute
    def forward(self, x, out: Optional[np.ndarray] = None) -> np.ndarray:
        x = _as_f32(x)
        B = x.shape[0]
        if out is None:
            out = np.empty((B, 51), np.float32)
        self._check(self.lib.lcn_forward(self.h, x.ctypes.data, out.ctypes.data, B, 0))
        return out

    def forward_loss(self, x, labels):
        x, labels = _as_f32(x), _as_f32(labels)
        B = x.shape[0]
        out = np.empty((B, 51), np.float32)
        loss = ctypes.c_float()
        self._check(self.lib.lcn_forward_loss(self.h, x.ctypes.data, labels.ctypes.data,
                                              out.ctypes.data, B, 0, ctypes.byref(loss)))
        return out, loss.value

    def train_step(self, x, labels, *, update=True, keep_grads=False, want_loss=True):
        x, labels = _as_f32(x), _as_f32(labels)
        flags = (0 if update else NO_UPDATE) | (KEEP_GRADS if keep_grads else 0)
        loss, lr = ctypes.c_float(), ctypes.c_float()
        self._check(self.lib.lcn_train_step(self.h, x.ctypes.data, labels.ctypes.data, x.shape[0],
                                            flags, ctypes.byref(loss) if want_loss else None,
                                            ctypes.byref(lr)))
        return (loss.value if want_loss else None), lr.value

    def train_step_device(self, x_ptr: int, lab_ptr: int, batch: int, *, sync=False):
        """One step on device-resident inputs (no host copies, no readback)."""
        flags = IN_DEVICE | (0 if sync else ASYNC)
        self._check(self.lib.lcn_train_step(self.h, x_ptr, lab_ptr, batch, flags, None, None))

    def forward_device(self, x_ptr: int, out_ptr: int, batch: int, *, sync=False):
        flags = IN_DEVICE | OUT_DEVICE | (0 if sync else ASYNC)
        self._check(self.lib.lcn_forward(self.h, x_ptr, out_ptr, batch, flags))

    def synchronize(self):
        self._check(self.lib.lcn_synchronize(self.h))

    def device_buffer(self, slot: int, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, slot, nbytes)

    # -- device-resident datasets
    def dataset_upload(self, slot: int, data: np.ndarray):
        """Keep `data` ([N][cols], float32 or float64 -- kept as given) in HBM."""
        a = np.asarray(data)
        if a.dtype not in (np.float32, np.float64):
            a = a.astype(np.float64)
        a = np.ascontiguousarray(a.reshape(a.shape[0], -1))
        dt = DTYPE_F64 if a.dtype == np.float64 else DTYPE_F32
        self._check(self.lib.lcn_dataset_upload(self.h, slot, a.ctypes.data, dt, a.shape[0],
                                                a.shape[1]))

    def dataset_free(self, slot: int):
        self._check(self.lib.lcn_dataset_free(self.h, slot))

    def train_step_indexed(self, x_slot: int, lab_slot: int, idx, *, update=True,
                           keep_grads=False, want_loss=True, idx_device_ptr: Optional[int] = None,
                           batch: Optional[int] = None, sync=True):
        """fit's step on dataset rows idx (host int array, or a device int32
        pointer + batch)."""
        flags = (0 if update else NO_UPDATE) | (KEEP_GRADS if keep_grads else 0)
        flags |= 0 if sync else ASYNC
        if idx_device_ptr is not None:
            ptr, B = idx_device_ptr, int(batch)
            flags |= IN_DEVICE
        else:
            ix = np.ascontiguousarray(idx, dtype=np.int32)
            ptr, B = ix.ctypes.data, ix.size
        loss, lr = ctypes.c_float(), ctypes.c_float()
        self._check(self.lib.lcn_train_step_indexed(
            self.h, x_slot, lab_slot, ptr, B, flags,
            ctypes.byref(loss) if (want_loss and sync) else None, ctypes.byref(lr)))
        return (loss.value if (want_loss and sync) else None), lr.value

    def predict_dataset(self, x_slot: int, n_rows: int, batch_size: int, *, lab_slot: int = -1,
                        augment=None, undo=None):
        """predict over a resident dataset; returns float64 [N][51] (and the
        per-batch float32 losses when lab_slot >= 0)."""
        out = np.empty((n_rows, 51), np.float64)
        nb_cap = max(1, -(-n_rows // batch_size)) if lab_slot >= 0 else 0
        losses = np.zeros(max(nb_cap, 1), np.float32)
        nb = ctypes.c_int64()
        a = make_augment(augment) if augment else None
        u = make_augment(undo) if undo else None
        self._check(self.lib.lcn_predict_dataset(
            self.h, x_slot, lab_slot, batch_size, ctypes.byref(a) if a else None,
            ctypes.byref(u) if u else None, out.ctypes.data_as(_f64p), n_rows,
            _fp(losses) if lab_slot >= 0 else None, nb_cap, ctypes.byref(nb)))
        if lab_slot >= 0:
            return out, losses[:nb.value]
        return out

    # -- data parallel
    @staticmethod
    def comm_unique_id() -> bytes:
        lib = load_library()
        buf = ctypes.create_string_buffer(128)
        rc = lib.lcn_comm_unique_id(buf)
        if rc != 0:
            raise LcnNativeError(f"lcn_comm_unique_id: {lib.lcn_last_error(None).decode()}")
        return buf.raw

    def comm_init(self, uid: bytes, rank: int, world: int):
        buf = ctypes.create_string_buffer(uid, 128)
        self._check(self.lib.lcn_comm_init(self.h, buf, rank, world))

    def comm_init_host(self, rank: int, world: int, allreduce):
        """Data parallel over a transport of the caller's (lcn_comm_init_host):
        allreduce(array, op) reduces the 1-D float32 / float64 numpy array in
        place over the ranks (op "sum" or "max") -- e.g. a gloo all_reduce of a
        CPU tensor sharing the array's memory.  An exception inside it fails
        the running liblcn call with LCN_E_COMM."""
        def cb(_ctx, buf, count, dtype, op):
            try:
                ct = ctypes.c_double if dtype == DTYPE_F64 else ctypes.c_float
                arr = np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(ct)), shape=(int(count),))
                allreduce(arr, "max" if op == 1 else "sum")
                return 0
            except Exception:  # noqa: BLE001 -- must not propagate through the C frame
                import traceback
                traceback.print_exc()
                return -1
        self._host_cb = HOST_ALLREDUCE_FN(cb)  # keep the thunk alive as long as the handle
        self._check(self.lib.lcn_comm_init_host(self.h, rank, world, self._host_cb, None))

    def comm_suspend(self, suspend: bool = True):
        """Run the following compute calls rank-locally (lcn_comm_suspend)."""
        self._check(self.lib.lcn_comm_suspend(self.h, int(bool(suspend))))

    def allreduce_host(self, values, op="sum") -> np.ndarray:
        v = np.ascontiguousarray(values, dtype=np.float64).copy()
        self._check(self.lib.lcn_comm_allreduce_host(self.h, v.ctypes.data_as(_f64p), v.size,
                                                     1 if op == "max" else 0))
        return v

    def comm_info(self):
        """(kind, rank, world) of the handle's communicator as it reports them
        itself (lcn_comm_info): kind "none" / "rccl" / "host"."""
        k, r, w = _i32(), _i32(), _i32()
        self._check(self.lib.lcn_comm_info(self.h, ctypes.byref(k), ctypes.byref(r), ctypes.byref(w)))
        return ("none", "rccl", "host")[k.value], r.value, w.value

    # -- instrumentation
    def set_dropout(self, rate: float, seed: int = 0):
        """tf.nn.dropout(rate) in training steps (lcn_set_dropout); 0 = off.
        The step counter of the masks restarts at 0."""
        self._check(self.lib.lcn_set_dropout(self.h, float(rate), int(seed) & (2 ** 64 - 1)))

    def set_timing(self, enable, only=None):
        """HIP-event timers around the kernel classes K_*: all of them, or
        only the classes listed in `only`; resets the accumulated timings."""
        flags = int(bool(enable))
        if enable and only is not None:
            flags = sum(1 << (1 + k) for k in only)
        self._check(self.lib.lcn_set_timing(self.h, flags))

    def kernel_timing(self, kernel: int):
        n, ms, fl = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        self._check(self.lib.lcn_kernel_timing(self.h, kernel, ctypes.byref(n), ctypes.byref(ms),
                                               ctypes.byref(fl)))
        return n.value, ms.value, fl.value

    def debug_tensor(self, kind: int, idx: int, n: int) -> np.ndarray:
        out = np.empty(n, np.float32)
        self._check(self.lib.lcn_debug_tensor(self.h, kind, idx, _fp(out), n))
        return out
