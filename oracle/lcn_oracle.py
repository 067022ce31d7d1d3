"""CPU oracle for the LCN hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity checker for the MI355X implementation in
``lcn-pose_amd/``.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it.  The product path never
routes through it (``lcn_amd.native`` raises if the HIP library is missing).

It is a plain-numpy restatement of the reference's locally-connected network
(adgx/lcn-pose, ``network/models_att.py``).  Each function cites the reference
lines it follows.  The reference executes its graph in TensorFlow 2.13.0, which
is not vendored and not installed here, so the op semantics below restate TF's
documented behaviour:

* ``tf.clip_by_norm(t, 1)``       -> ``t * 1 / max(||t||_F, 1)``  (division, as TF)
* ``tf.nn.softmax(V, axis=0)``    -> ``exp(V - max) / sum``
* Keras ``BatchNormalization``    -> ``tf.nn.moments`` (two-pass, biased variance) and
  ``tf.nn.batch_normalization``: ``inv = rsqrt(var + eps) * gamma``;
  ``u = z * inv + (beta - mean * inv)``; eps = 1e-3; always batch statistics
  (``training=self.is_training`` and ``is_training=True`` is hard-wired,
  models_att.py:528, 667, 696, 737; train.py:107 -> params_help.py:170).
* ``tf.nn.leaky_relu``            -> ``x > 0 ? x : 0.2 * x``
* ``tf.nn.dropout(rate=0)``       -> identity
* ``tf.compat.v1.train.AdamOptimizer`` (ApplyAdam kernel):
  ``alpha = lr * sqrt(1 - b2^t) / (1 - b1^t)``; ``m += (g - m)(1 - b1)``;
  ``v += (g^2 - v)(1 - b2)``; ``theta -= m * alpha / (sqrt(v) + eps)``
* ``tf.compat.v1.train.exponential_decay(staircase=False)``:
  ``lr * rate ** (global_step / decay_steps)`` in float32.

Parity status: the arithmetic of the TF graph is **unpinned** (TF absent, no
reference checkpoint or golden output exists).  The oracle is pinned on
everything the reference itself can produce here: the knn neighbour matrices
(reference helper + Kaggle notebook outputs), the exponential mask
(reference helper), the flip/rotate/undo TTA helpers (reference helpers), the
learning-rate schedule (values printed in the notebook logs); and it is
cross-checked against float64 finite differences and torch autograd
(``tests/test_oracle.py``).

Layouts (joint-major, as the reference): activations ``a[b, j*F + f]``,
input ``x[b, 2*j + c]``, output ``out[b, 3*j + c]``; weights ``W[i*Fin + p,
j*Fout + q]`` with ``i`` the input joint and ``j`` the output joint
(models_att.py:582).
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional, Tuple

import numpy as np

J = 17

# tools/filter_hub.py:4-24 -- the H36M 17-joint skeleton adjacency.
NEIGHBOUR_DICT = {
    0: [1, 4, 7], 1: [0, 7, 2], 2: [1, 3], 3: [2], 4: [0, 7, 5], 5: [4, 6],
    6: [5], 7: [1, 0, 4, 14, 8, 11], 8: [7, 9, 11, 14], 9: [8, 10], 10: [9],
    11: [8, 7, 12], 12: [11, 13], 13: [12], 14: [8, 7, 15], 15: [14, 16],
    16: [15],
}

# models_att.py:19-36 -- the edge list of get_exponential_matrix (18 edges; it
# lacks 8-11 and 8-14 compared with filter_hub, which is reproduced as is).
EXP_EDGES = [(0, 1), (0, 7), (0, 4), (4, 5), (4, 7), (5, 6), (1, 7), (1, 2),
             (2, 3), (7, 11), (7, 8), (7, 14), (11, 12), (12, 13), (14, 15),
             (15, 16), (8, 9), (9, 10)]


def neighbour_matrix(knn: int = 1) -> np.ndarray:
    """tools/params_help.py:8-20 (get_neighbour_matrix_by_hand)."""
    n = np.zeros((J, J), dtype=np.float32)
    for idx in range(J):
        n[idx, [idx] + NEIGHBOUR_DICT[idx]] = 1
    if knn >= 2:
        n = np.linalg.matrix_power(n, knn)
        n = np.array(n != 0, dtype=np.float32)
    return n


def exponential_matrix() -> np.ndarray:
    """models_att.py:14-69 (get_exponential_matrix), without its prints."""
    dist = np.full((J, J), np.inf)
    np.fill_diagonal(dist, 0)
    for u, v in EXP_EDGES:
        dist[u][v] = 1
        dist[v][u] = 1
    for k in range(J):
        for i in range(J):
            for j in range(J):
                if dist[i, j] > dist[i, k] + dist[k, j]:
                    dist[i, j] = dist[i, k] + dist[k, j]
    return (1 / (2 ** dist)).astype(np.float32)


@dataclasses.dataclass
class Config:
    """Subset of cgcnn(**params) (models_att.py:478-532) that shapes the math."""
    F: int = 64
    in_F: int = 2
    num_layers: int = 3
    mask_type: str = "locally_connected"
    neighbour: Optional[np.ndarray] = None      # [17,17]; LC structure N
    residual: bool = True
    batch_norm: bool = True
    max_norm: bool = True
    regularization: Optional[float] = 0.0
    learning_rate: float = 1e-3
    decay_steps: int = 32000
    decay_rate: float = 0.96
    bn_eps: float = 1e-3
    leaky_alpha: float = 0.2
    beta1: float = 0.9
    beta2: float = 0.999
    adam_eps: float = 1e-8

    @property
    def learnable_mask(self) -> bool:
        return "locally_connected" in self.mask_type

    @property
    def H(self) -> int:
        return J * self.F


def param_specs(cfg: Config) -> List[Tuple[str, Tuple[int, ...]]]:
    """Canonical parameter order = TF variable creation order.

    mask (models_att.py:557) -> w1, b1 (:714, :721) -> BN0 gamma/beta (:736) ->
    per block l: w2_l, b2_l, BN1l, w3_l, b3_l, BN2l (:647-698) -> w4, b4 (:750-761).
    Only trainable variables are listed (BN moving statistics are never used,
    because BN always runs in training mode).
    """
    H, F, in_F = cfg.H, cfg.F, cfg.in_F
    specs: List[Tuple[str, Tuple[int, ...]]] = []
    if cfg.learnable_mask:
        specs.append(("mask", (J, J)))
    specs += [("w1", (J * in_F, H)), ("b1", (H,))]
    if cfg.batch_norm:
        specs += [("bn0_gamma", (F,)), ("bn0_beta", (F,))]
    for l in range(cfg.num_layers):
        specs += [(f"w2_{l}", (H, H)), (f"b2_{l}", (H,))]
        if cfg.batch_norm:
            specs += [(f"bn1{l}_gamma", (F,)), (f"bn1{l}_beta", (F,))]
        specs += [(f"w3_{l}", (H, H)), (f"b3_{l}", (H,))]
        if cfg.batch_norm:
            specs += [(f"bn2{l}_gamma", (F,)), (f"bn2{l}_beta", (F,))]
    specs += [("w4", (H, J * 3)), ("b4", (J * 3,))]
    return specs


def layer_names(cfg: Config) -> List[Tuple[str, str, Optional[str], int, int]]:
    """(weight, bias, bn-prefix, Fin, Fout) per linear layer, in forward order."""
    out = [("w1", "b1", "bn0" if cfg.batch_norm else None, cfg.in_F, cfg.F)]
    for l in range(cfg.num_layers):
        out.append((f"w2_{l}", f"b2_{l}", f"bn1{l}" if cfg.batch_norm else None, cfg.F, cfg.F))
        out.append((f"w3_{l}", f"b3_{l}", f"bn2{l}" if cfg.batch_norm else None, cfg.F, cfg.F))
    out.append(("w4", "b4", None, cfg.F, 3))
    return out


def truncated_normal(rng: np.random.Generator, shape) -> np.ndarray:
    """tf.random.truncated_normal(mean 0, stddev 1): redraw outside 2 sigma."""
    out = rng.standard_normal(size=shape)
    bad = np.abs(out) > 2.0
    while bad.any():
        out[bad] = rng.standard_normal(size=int(bad.sum()))
        bad = np.abs(out) > 2.0
    return out


def init_params(cfg: Config, seed: int = 0) -> Dict[str, np.ndarray]:
    """cgcnn.kaiming (models_att.py:614-628): trunc_normal * sqrt(2/shape[0]).

    Biases use shape[0] = len(b).  The mask starts at N^T (init_type 'same',
    :549-566); BN gamma = 1, beta = 0 (Keras defaults).
    """
    rng = np.random.default_rng(seed)
    p: Dict[str, np.ndarray] = {}
    for name, shape in param_specs(cfg):
        if name == "mask":
            p[name] = np.array(cfg.neighbour, dtype=np.float32).T.copy()
        elif name.endswith("_gamma"):
            p[name] = np.ones(shape, np.float32)
        elif name.endswith("_beta"):
            p[name] = np.zeros(shape, np.float32)
        else:
            p[name] = (truncated_normal(rng, shape) * math.sqrt(2.0 / shape[0])).astype(np.float32)
    return p


def flatten(cfg: Config, params: Dict[str, np.ndarray]) -> np.ndarray:
    return np.concatenate([np.asarray(params[n], np.float32).ravel() for n, _ in param_specs(cfg)])


def unflatten(cfg: Config, flat: np.ndarray) -> Dict[str, np.ndarray]:
    out, off = {}, 0
    for n, shape in param_specs(cfg):
        size = int(np.prod(shape))
        out[n] = flat[off:off + size].reshape(shape)
        off += size
    assert off == flat.size
    return out


# ----------------------------------------------------------------------------
# Mask and weight preparation
# ----------------------------------------------------------------------------

def structure(cfg: Config) -> np.ndarray:
    """C = 1[L != 0] with L = N^T (models_att.py:549, 571); row i = input joint."""
    if cfg.learnable_mask:
        return (np.asarray(cfg.neighbour).T != 0).astype(np.float32)
    return np.ones((J, J), np.float32)


def mask_value(cfg: Config, params, dtype=np.float32) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """models_att.py:547-574.  Returns (M, S) with S = softmax(V, 0) (LC only)."""
    if cfg.learnable_mask:
        V = params["mask"].astype(dtype)
        e = np.exp(V - V.max(axis=0, keepdims=True))
        S = e / e.sum(axis=0, keepdims=True)
        return S * structure(cfg).astype(dtype), S
    return exponential_matrix().astype(dtype), None


def effective_weight(cfg: Config, W: np.ndarray, M: np.ndarray, Fin: int, Fout: int):
    """clip_by_norm (models_att.py:659/690/726/762) then mask_weights (:576-586).

    Returns (W_e, W_c, norm)."""
    n = np.sqrt(np.sum(W * W, dtype=W.dtype))
    if cfg.max_norm:
        Wc = (W * W.dtype.type(1)) / max(n, W.dtype.type(1))
    else:
        Wc = W
    We = (Wc.reshape(J, Fin, J, Fout) * M.reshape(J, 1, J, 1)).reshape(W.shape)
    return We, Wc, n


# ----------------------------------------------------------------------------
# Forward
# ----------------------------------------------------------------------------

def _bn_forward(cfg: Config, z, gamma, beta, F):
    """batch_normalization_warp (models_att.py:588-612) in training mode."""
    B = z.shape[0]
    z3 = z.reshape(B, J, F)
    mean = z3.mean(axis=(0, 1))
    var = ((z3 - mean) ** 2).mean(axis=(0, 1))
    rstd = 1.0 / np.sqrt(var + z.dtype.type(cfg.bn_eps))
    inv = rstd * gamma
    u = z3 * inv + (beta - mean * inv)
    return u.reshape(B, -1), dict(mean=mean, var=var, rstd=rstd, inv=inv)


def _act(cfg, u):
    return np.where(u > 0, u, u * u.dtype.type(cfg.leaky_alpha))


def _fmix32(x):
    x = np.asarray(x, np.uint32)
    x = x ^ (x >> np.uint32(16))
    x = x * np.uint32(0x85EBCA6B)
    x = x ^ (x >> np.uint32(13))
    x = x * np.uint32(0xC2B2AE35)
    return x ^ (x >> np.uint32(16))


def dropout_mask(rate, seed, step, k, B, H, row0=0):
    """Keep mask [B, H] of BN layer k's dropout in training step ``step``
    after lcn_set_dropout(rate, seed) -- the counter-based hash of
    lcn_internal.h (Dropout, drop_keep) and lcn_api.cpp (run_train_step,
    drop_of).  Not TF's random stream (which cannot be reproduced); TF's
    dropout semantics (models_att.py:673, 700, 742): keep iff u >= rate with
    u uniform in [0, 1), kept values scaled by float32(1 / (1 - rate))."""
    with np.errstate(over="ignore"):
        s32 = np.uint32((int(seed) ^ (int(seed) >> 32)) & 0xFFFFFFFF)
        step_seed = _fmix32(s32 + _fmix32(np.uint32((step + 0x9E3779B9) & 0xFFFFFFFF)))
        lseed = _fmix32(step_seed ^ np.uint32(((k + 1) * 0x9E3779B9) & 0xFFFFFFFF))
        key = ((np.arange(B, dtype=np.uint64)[:, None] + np.uint64(row0)) * np.uint64(H)
               + np.arange(H, dtype=np.uint64)[None, :])
        lo = (key & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi = (key >> np.uint64(32)).astype(np.uint32)
        xh = _fmix32(_fmix32(lo ^ lseed) + hi)
    u = (xh >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)
    return u >= np.float32(rate)


def dropout_scale(rate):
    """TF: 1 / (1 - rate) in float32."""
    return np.float32(1) / (np.float32(1) - np.float32(rate))


def forward(cfg: Config, params, x: np.ndarray, dtype=np.float32, keep: bool = True,
            drop: Optional[Tuple[float, int, int]] = None):
    """_inference_lcn (models_att.py:707-775).  Returns (out, cache).

    ``drop`` = (rate, seed, step): the training graph's tf.nn.dropout after
    every BN + LeakyReLU (models_att.py:673, 700, 742) with the masks of
    dropout_mask."""
    P = {k: np.asarray(v, dtype) for k, v in params.items()}
    x = np.asarray(x, dtype)
    B = x.shape[0]
    M, S = mask_value(cfg, P, dtype)
    layers = layer_names(cfg)
    eff = {}
    for (wn, bn, bnp, fin, fout) in layers:
        eff[wn] = effective_weight(cfg, P[wn], M, fin, fout)
    cache = dict(M=M, S=S, eff=eff, x=x, layers=[])

    def linear_bn_act(a, li):
        wn, bname, bnp, fin, fout = layers[li]
        z = a @ eff[wn][0] + P[bname]
        if bnp is not None:
            u, st = _bn_forward(cfg, z, P[bnp + "_gamma"], P[bnp + "_beta"], fout)
        else:
            u, st = z, None
        h = _act(cfg, u)
        m = None
        if drop is not None and drop[0] > 0:
            m = dropout_mask(drop[0], drop[1], drop[2], li, B, fout * J)
            h = np.where(m, h * h.dtype.type(dropout_scale(drop[0])), h.dtype.type(0))
        if keep:
            cache["layers"].append(dict(a=a, z=z, u=u, st=st, m=m,
                                        scale=dropout_scale(drop[0]) if m is not None else None))
        return h, z, st

    h, _, _ = linear_bn_act(x, 0)                          # :729-742
    li = 1
    block_in = []
    for l in range(cfg.num_layers):                        # :745-746
        hin = h
        g, _, _ = linear_bn_act(hin, li)                   # :662-673
        t, _, _ = linear_bn_act(g, li + 1)                 # :692-700
        h = hin + t if cfg.residual else t                 # :704
        block_in.append(hin)
        li += 2
    wn, bname, _, _, _ = layers[-1]
    y = h @ eff[wn][0] + P[bname]                          # :765
    if keep:
        cache["hL"] = h
        cache["block_in"] = block_in
    x3 = x.reshape(B, J, cfg.in_F)
    y3 = y.reshape(B, J, 3)
    out = np.concatenate([x3[:, :, :2] + y3[:, :, :2], y3[:, :, 2:3]], axis=2)  # :768-773
    return out.reshape(B, J * 3), cache


def mse_loss(out: np.ndarray, lab: np.ndarray) -> float:
    """base_model.loss (models_att.py:356)."""
    d = out - np.asarray(lab, out.dtype)
    return float(np.mean(d * d))


def reg_loss(cfg: Config, params, dtype=np.float64) -> float:
    """models_att.py:362-365 + _variable (:465-472): reg * sum(l2_loss(W, b))."""
    if cfg.regularization in (0, None):
        return 0.0
    tot = 0.0
    for (wn, bn, _, _, _) in layer_names(cfg):
        tot += float(np.sum(np.asarray(params[wn], dtype) ** 2) / 2)
        tot += float(np.sum(np.asarray(params[bn], dtype) ** 2) / 2)
    return cfg.regularization * tot


# ----------------------------------------------------------------------------
# Backward (analytic)
# ----------------------------------------------------------------------------

def _bn_act_backward(cfg, dh, rec, F, gamma, pos=None):
    """``pos`` (test hook): the LeakyReLU branch mask u > 0 to use instead of
    this pass's own -- a float32 forward whose u lands on the other side of 0
    than the float64 one takes the other branch of the kink."""
    B = dh.shape[0]
    u = rec["u"]
    if rec.get("m") is not None:  # tf.nn.dropout's gradient: dh * mask * scale
        dh = np.where(rec["m"], dh * dh.dtype.type(rec["scale"]), dh.dtype.type(0))
    if pos is None:
        pos = u > 0
    du = dh * np.where(pos, dh.dtype.type(1), dh.dtype.type(cfg.leaky_alpha))
    st = rec["st"]
    if st is None:
        return du, None, None
    N = B * J
    z3 = rec["z"].reshape(B, J, F)
    zhat = (z3 - st["mean"]) * st["rstd"]
    du3 = du.reshape(B, J, F)
    S1 = du3.sum(axis=(0, 1))
    S2 = (du3 * zhat).sum(axis=(0, 1))
    dz = (gamma * st["rstd"] / N) * (N * du3 - S1 - zhat * S2)
    return dz.reshape(B, -1), S2, S1


def backward(cfg: Config, params, cache, lab: np.ndarray, dtype=np.float32,
             global_batch: Optional[int] = None,
             kinks: Optional[Dict[int, np.ndarray]] = None) -> Dict[str, np.ndarray]:
    """Gradients of the MSE loss (+ regularisation) w.r.t. every trainable.

    ``global_batch`` lets a shard scale its loss gradient by the global batch
    (data-parallel decomposition tests).  ``kinks`` maps a linear layer index
    to the [B, H] mask u > 0 to differentiate LeakyReLU with (tests compare a
    float32 device run against float64 at the device's own kink branches)."""
    kinks = kinks or {}
    P = {k: np.asarray(v, dtype) for k, v in params.items()}
    layers = layer_names(cfg)
    eff = cache["eff"]
    B = cache["x"].shape[0]
    Bg = B if global_batch is None else global_batch
    out, _ = None, None
    hL = cache["hL"]
    wn4, bn4, _, _, _ = layers[-1]
    y = hL @ eff[wn4][0] + P[bn4]
    x3 = cache["x"].reshape(B, J, cfg.in_F)
    y3 = y.reshape(B, J, 3)
    out = np.concatenate([x3[:, :, :2] + y3[:, :, :2], y3[:, :, 2:3]], axis=2).reshape(B, -1)
    dy = (dtype(2.0) / dtype(Bg * J * 3)) * (out - np.asarray(lab, dtype))
    g: Dict[str, np.ndarray] = {}
    dWe = {}
    dWe[wn4] = hL.T @ dy
    g[bn4] = dy.sum(axis=0)
    dh = dy @ eff[wn4][0].T

    recs = cache["layers"]
    li = len(layers) - 2
    for l in reversed(range(cfg.num_layers)):
        dres = dh
        # second linear of block l (layer li)
        for k in (li, li - 1):
            wn, bname, bnp, fin, fout = layers[k]
            rec = recs[k]
            gamma = P[bnp + "_gamma"] if bnp else None
            dz, dgam, dbet = _bn_act_backward(cfg, dh, rec, fout, gamma, kinks.get(k))
            if bnp:
                g[bnp + "_gamma"], g[bnp + "_beta"] = dgam, dbet
            dWe[wn] = rec["a"].T @ dz
            g[bname] = dz.sum(axis=0)
            dh = dz @ eff[wn][0].T
        if cfg.residual:
            dh = dh + dres
        li -= 2
    wn, bname, bnp, fin, fout = layers[0]
    rec = recs[0]
    gamma = P[bnp + "_gamma"] if bnp else None
    dz, dgam, dbet = _bn_act_backward(cfg, dh, rec, fout, gamma, kinks.get(0))
    if bnp:
        g[bnp + "_gamma"], g[bnp + "_beta"] = dgam, dbet
    dWe[wn] = rec["a"].T @ dz
    g[bname] = dz.sum(axis=0)

    # mask / clip backward
    M, S = cache["M"], cache["S"]
    dM = np.zeros((J, J), dtype)
    for (wn, bname, _, fin, fout) in layers:
        We, Wc, n = eff[wn]
        d4 = dWe[wn].reshape(J, fin, J, fout)
        dWc = (d4 * M.reshape(J, 1, J, 1)).reshape(We.shape)
        dM += (d4 * Wc.reshape(J, fin, J, fout)).sum(axis=(1, 3))
        W = P[wn]
        if cfg.max_norm and n > 1:
            dW = dWc / n - (np.sum(dWc * W) / (n ** 3)) * W
        else:
            dW = dWc
        g[wn] = dW
    if cfg.regularization not in (0, None):
        for (wn, bname, _, _, _) in layers:
            g[wn] = g[wn] + dtype(cfg.regularization) * P[wn]
            g[bname] = g[bname] + dtype(cfg.regularization) * P[bname]
    if cfg.learnable_mask:
        C = structure(cfg).astype(dtype)
        dS = dM * C
        g["mask"] = S * (dS - (S * dS).sum(axis=0, keepdims=True))
    return {k: np.asarray(v, dtype) for k, v in g.items()}


# ----------------------------------------------------------------------------
# Data-parallel decomposition (SyncBN), as liblcn runs it with world > 1
# ----------------------------------------------------------------------------

def _tile_moments(z3: np.ndarray, tile_rows: int = 128):
    """Per-channel (sum z, sum (M2_t + s_t^2 / n_t)) over the 128-row groups of a
    shard -- the float64 quantities bn_fwd_finalize all-reduces
    (lcn-pose_amd/csrc/kernels_elem.hip colreduce mode 1)."""
    B, _, F = z3.shape
    S = np.zeros(F)
    Q = np.zeros(F)
    for r0 in range(0, B, tile_rows):
        t = z3[r0:r0 + tile_rows].astype(np.float64)          # [n, J, F]
        for j in range(J):
            col = t[:, j, :]
            s = col.sum(axis=0)
            m2 = ((col - s / col.shape[0]) ** 2).sum(axis=0)
            S += s
            Q += m2 + s * s / col.shape[0]
    return S, Q


def sharded_grads(cfg: Config, params, x: np.ndarray, lab: np.ndarray, allreduce,
                  world: int, dtype=np.float64):
    """One rank's view of a data-parallel step: forward with SyncBN statistics
    (per-shard tile moments -> all-reduce -> mean / biased variance), backward
    with all-reduced BN-backward sums, LOCAL raw gradients (dW_e, db, dgamma,
    dbeta) summed over ranks by one all-reduce, then the mask / clip backward
    on the global raw gradient.  ``allreduce(a)`` returns the elementwise sum of
    ``a`` over ranks.  Equals ``backward(forward(full batch))`` -- the identity
    tests/test_distributed.py checks over gloo.  Follows the same reference
    lines as forward/backward (models_att.py:588-612, 707-775, :356)."""
    P = {k: np.asarray(v, dtype) for k, v in params.items()}
    x = np.asarray(x, dtype)
    B = x.shape[0]
    Bg = int(allreduce(np.array([float(B)]))[0])
    M, S_mask = mask_value(cfg, P, dtype)
    layers = layer_names(cfg)
    eff = {wn: effective_weight(cfg, P[wn], M, fin, fout) for (wn, _, _, fin, fout) in layers}
    recs = []

    def lin(a, li):
        wn, bname, bnp, fin, fout = layers[li]
        z = a @ eff[wn][0] + P[bname]
        st = None
        if bnp is not None:
            z3 = z.reshape(B, J, fout)
            S1, Q = _tile_moments(z3)
            tot = allreduce(np.concatenate([S1, Q]))
            N = Bg * J
            mean = tot[:fout] / N
            var = np.maximum(tot[fout:] / N - mean * mean, 0.0)
            rstd = 1.0 / np.sqrt(var + cfg.bn_eps)
            inv = rstd * P[bnp + "_gamma"]
            u = (z3 * inv + (P[bnp + "_beta"] - mean * inv)).reshape(B, -1)
            st = dict(mean=mean, rstd=rstd)
        else:
            u = z
        recs.append(dict(a=a, z=z, u=u, st=st))
        return _act(cfg, u)

    h = lin(x, 0)
    li = 1
    for _ in range(cfg.num_layers):
        hin = h
        t = lin(lin(hin, li), li + 1)
        h = hin + t if cfg.residual else t
        li += 2
    wn4, bn4, _, _, _ = layers[-1]
    y = h @ eff[wn4][0] + P[bn4]
    x3 = x.reshape(B, J, cfg.in_F)
    y3 = y.reshape(B, J, 3)
    out = np.concatenate([x3[:, :, :2] + y3[:, :, :2], y3[:, :, 2:3]], axis=2).reshape(B, -1)
    dy = (2.0 / (Bg * J * 3)) * (out - np.asarray(lab, dtype))     # global-mean loss
    raw = {wn4: h.T @ dy, bn4: dy.sum(axis=0)}
    dh = dy @ eff[wn4][0].T

    def bn_back(dh, k):
        wn, bname, bnp, fin, fout = layers[k]
        rec = recs[k]
        du = dh * np.where(rec["u"] > 0, 1.0, cfg.leaky_alpha)
        if rec["st"] is None:
            dz = du
        else:
            st = rec["st"]
            z3 = rec["z"].reshape(B, J, fout)
            zhat = (z3 - st["mean"]) * st["rstd"]
            du3 = du.reshape(B, J, fout)
            loc = np.concatenate([du3.sum(axis=(0, 1)), (du3 * zhat).sum(axis=(0, 1))])
            tot = allreduce(loc)                                    # c123 from global sums
            N = Bg * J
            c1 = P[bnp + "_gamma"] * st["rstd"]
            c3 = -c1 * st["rstd"] * tot[fout:] / N
            c2 = -c1 * tot[:fout] / N - c3 * st["mean"]
            dz = (c1 * du3 + c2 + c3 * z3).reshape(B, -1)
            raw[bnp + "_beta"] = loc[:fout]                         # local contributions
            raw[bnp + "_gamma"] = loc[fout:]
        raw[wn] = rec["a"].T @ dz
        raw[bname] = dz.sum(axis=0)
        return dz @ eff[wn][0].T

    li = len(layers) - 2
    for _ in range(cfg.num_layers):
        dres = dh
        dh = bn_back(bn_back(dh, li), li - 1)
        if cfg.residual:
            dh = dh + dres
        li -= 2
    bn_back(dh, 0)

    names = sorted(raw)
    flat = allreduce(np.concatenate([raw[n].ravel() for n in names]))
    g, o = {}, 0
    for n in names:
        g[n] = flat[o:o + raw[n].size].reshape(raw[n].shape)
        o += raw[n].size
    # mask / clip backward and regularisation on the global raw gradient
    dM = np.zeros((J, J), dtype)
    for (wn, bname, _, fin, fout) in layers:
        We, Wc, n = eff[wn]
        d4 = g[wn].reshape(J, fin, J, fout)
        dWc = (d4 * M.reshape(J, 1, J, 1)).reshape(We.shape)
        dM += (d4 * Wc.reshape(J, fin, J, fout)).sum(axis=(1, 3))
        W = P[wn]
        g[wn] = dWc / n - (np.sum(dWc * W) / (n ** 3)) * W if (cfg.max_norm and n > 1) else dWc
    if cfg.regularization not in (0, None):
        for (wn, bname, _, _, _) in layers:
            g[wn] = g[wn] + cfg.regularization * P[wn]
            g[bname] = g[bname] + cfg.regularization * P[bname]
    if cfg.learnable_mask:
        dS = dM * structure(cfg).astype(dtype)
        g["mask"] = S_mask * (dS - (S_mask * dS).sum(axis=0, keepdims=True))
    return out, g


# ----------------------------------------------------------------------------
# Optimiser
# ----------------------------------------------------------------------------

def learning_rate(cfg: Config, global_step: int) -> np.float32:
    """exponential_decay(lr, global_step, 32000, 0.96, staircase=False)
    (models_att.py:392-399, params_help.py:129-130), float32 arithmetic."""
    p = np.float32(global_step) / np.float32(cfg.decay_steps)
    return np.float32(np.float32(cfg.learning_rate) * np.power(np.float32(cfg.decay_rate), p))


@dataclasses.dataclass
class AdamState:
    m: Dict[str, np.ndarray]
    v: Dict[str, np.ndarray]
    global_step: int = 0
    beta1_power: np.float32 = np.float32(0.9)
    beta2_power: np.float32 = np.float32(0.999)


def adam_init(cfg: Config, params) -> AdamState:
    return AdamState({k: np.zeros_like(v, np.float32) for k, v in params.items()},
                     {k: np.zeros_like(v, np.float32) for k, v in params.items()},
                     0, np.float32(cfg.beta1), np.float32(cfg.beta2))


def adam_step(cfg: Config, params, grads, st: AdamState):
    """AdamOptimizer.apply_gradients (models_att.py:404-409), in place.

    Returns the learning rate used (what op_train returns, :419-420)."""
    lr = learning_rate(cfg, st.global_step)
    b1, b2, eps = np.float32(cfg.beta1), np.float32(cfg.beta2), np.float32(cfg.adam_eps)
    alpha = np.float32(lr * np.sqrt(np.float32(1) - st.beta2_power) / (np.float32(1) - st.beta1_power))
    for k in params:
        gk = np.asarray(grads[k], np.float32)
        m, v = st.m[k], st.v[k]
        m += (gk - m) * (np.float32(1) - b1)
        v += (gk * gk - v) * (np.float32(1) - b2)
        params[k] = (params[k] - (m * alpha) / (np.sqrt(v) + eps)).astype(np.float32)
    st.beta1_power = np.float32(st.beta1_power * b1)
    st.beta2_power = np.float32(st.beta2_power * b2)
    st.global_step += 1
    return lr


def train_step(cfg: Config, params, st: AdamState, x, lab, dtype=np.float32):
    """One op_train (models_att.py:382-421): forward, loss, grads, Adam."""
    out, cache = forward(cfg, params, x, dtype)
    loss = mse_loss(out, lab) + reg_loss(cfg, params)
    grads = backward(cfg, params, cache, lab, dtype)
    lr = adam_step(cfg, params, grads, st)
    return loss, lr, grads


# ----------------------------------------------------------------------------
# Test-time augmentation helpers (tools/data.py)
# ----------------------------------------------------------------------------

LEFT = [4, 5, 6, 11, 12, 13]
RIGHT = [1, 2, 3, 14, 15, 16]


def flip_data(data: np.ndarray) -> np.ndarray:
    """tools/data.py:10-25."""
    f = data.copy().reshape((len(data), J, -1))
    f[:, :, 0] *= -1
    f[:, LEFT + RIGHT] = f[:, RIGHT + LEFT]
    return f.reshape(data.shape)


def rotate_data(data: np.ndarray, angle: float = 180) -> np.ndarray:
    """tools/data.py:289-322 (2-D uses Rz.T[:2,:2]; 3-D rotates about joint 0)."""
    th = np.radians(angle)
    Rz = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]])
    r = data.copy().reshape((len(data), J, -1)).astype(np.float64)
    k = r.shape[2]
    piv = r[:, 0:1, :min(k, 3)].copy()
    if k == 2:
        r = (r - piv) @ Rz.T[:2, :2] + piv
    else:
        r[:, :, :3] = (r[:, :, :3] - piv) @ Rz.T + piv
    return r.reshape(data.shape).astype(data.dtype)


def translation_data(data: np.ndarray, translation_factor: float = 0.5) -> np.ndarray:
    """tools/data.py:27-54 (scalar factor): x, y (and a third channel) + t."""
    t = data.copy().reshape((len(data), J, -1))
    t[:, :, 0] += translation_factor
    t[:, :, 1] += translation_factor
    if t.shape[2] == 3:
        t[:, :, 2] += translation_factor
    return t.reshape(data.shape)


def undo(preds: np.ndarray, op_ord: dict, number_actions: int, angle: float = 180,
         translation: float = 0.5) -> np.ndarray:
    """tools/data.py:269-287 (unflip :236-249, rotate, untranslate :205-218)."""
    d = preds.copy().reshape(number_actions + 1, -1, J, 3)
    if "f" in op_ord:
        u = d[op_ord["f"]].copy()
        u[:, :, 0] *= -1
        u[:, LEFT + RIGHT] = u[:, RIGHT + LEFT]
        d[op_ord["f"]] = u
    if "r" in op_ord:
        d[op_ord["r"]] = rotate_data(d[op_ord["r"]], angle)
    if "t" in op_ord:
        d[op_ord["t"]] = d[op_ord["t"]] - translation
    return d.mean(axis=0).reshape(-1, J * 3)
