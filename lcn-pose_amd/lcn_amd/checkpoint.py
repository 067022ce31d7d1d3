"""Checkpoints in the reference's layout and TensorFlow's file format.

tf.compat.v1.train.Saver(max_to_keep=1) writes ``<dir>/model-<step>.index`` /
``.data-00000-of-00001`` (+ ``.meta``) and a ``checkpoint`` text file naming
the latest prefix (models_att.py:161-162, 256-260, 321-322);
tf.train.latest_checkpoint reads that file and Saver.restore the bundle
(:452-461).  ``save`` writes the same files through lcn_amd.tf_bundle under the
variable names the reference graph gives its variables (``tf_name_map``):

  mask                                         LC mask logits V (:557-566)
  linear_model/{w1,b1,w4,b4}                   lift / output layer (:717-761)
  linear_model/batch_normalization/{gamma,beta,moving_mean,moving_variance}
  linear_model/two_linear_<i>/{w2_<i>,b2_<i>,w3_<i>,b3_<i>}      (:630-705)
  linear_model/two_linear_<i>/batch_normalization{1,2}<i>/...    (:664-697)
  <var>/Adam, <var>/Adam_1                     AdamOptimizer slots m, v
  beta1_power, beta2_power, global_step        Adam / training state (:386-409)
  loss/{mse_loss/Mean,add}/ExponentialMovingAverage
                                               loss EMA(0.9) shadows (:368-379):
                                               zero-initialised, zero_debias off
                                               (the v1 default), so no /biased or
                                               /local_step companions exist

Keras BN moving statistics are written as their initial values (0, 1): the
reference never runs their update ops (it trains and predicts with batch
statistics, models_att.py:588-612).  These names follow TF1 / Keras naming
rules; they are unverified against a real TF checkpoint (none exists offline).
``restore`` reads these files, and the earlier ``.npz`` payload.
"""
from __future__ import annotations

import glob
import os
import re
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import tf_bundle


def _bn_scope(name: str) -> Tuple[str, str]:
    """our BN parameter name -> (TF layer scope, gamma|beta)."""
    m = re.fullmatch(r"bn(\d+)_(gamma|beta)", name)
    if not m:
        raise KeyError(name)
    tag, which = m.group(1), m.group(2)
    if tag == "0":
        return "linear_model/batch_normalization", which
    kind, idx = tag[0], tag[1:]                      # "1<idx>" / "2<idx>"
    return f"linear_model/two_linear_{idx}/batch_normalization{kind}{idx}", which


def tf_name_map(layout) -> List[Tuple[str, str, int, tuple]]:
    """(our name, TF variable name, offset, shape) per trainable variable."""
    out = []
    for name, off, shape in layout:
        if name == "mask":
            tf = "mask"
        elif name in ("w1", "b1", "w4", "b4"):
            tf = f"linear_model/{name}"
        elif re.fullmatch(r"[wb][23]_\d+", name):
            tf = f"linear_model/two_linear_{name.split('_')[1]}/{name}"
        else:
            scope, which = _bn_scope(name)
            tf = f"{scope}/{which}"
        out.append((name, tf, off, tuple(shape)))
    return out


def _ema_names(regularized: bool) -> Tuple[str, str]:
    # loss() ops (:353-366): "loss/mse_loss/Mean" and the total "loss/add"
    # ("loss/add_1" once the regularisation term is added)
    return "loss/mse_loss/Mean", ("loss/add_1" if regularized else "loss/add")


def to_tensors(net, loss_ema=None, regularized=False) -> Dict[str, np.ndarray]:
    params = net.get_params()
    m, v, gs, b1p, b2p = net.get_optimizer_state()
    t: Dict[str, np.ndarray] = {}
    for _, tf, off, shape in tf_name_map(net.param_layout()):
        n = int(np.prod(shape))
        t[tf] = params[off:off + n].reshape(shape).copy()
        t[tf + "/Adam"] = m[off:off + n].reshape(shape).copy()
        t[tf + "/Adam_1"] = v[off:off + n].reshape(shape).copy()
        if tf.endswith("/gamma"):
            scope = tf[:-len("/gamma")]
            t[scope + "/moving_mean"] = np.zeros(shape, np.float32)
            t[scope + "/moving_variance"] = np.ones(shape, np.float32)
    t["beta1_power"] = np.float32(b1p).reshape(())
    t["beta2_power"] = np.float32(b2p).reshape(())
    t["global_step"] = np.int32(gs).reshape(())
    # the shadow of a tensor starts at 0 and is never debiased (zero_debias=False)
    shadow = loss_ema[0] if loss_ema else 0.0
    for op in _ema_names(regularized):
        t[op + "/ExponentialMovingAverage"] = np.float32(shadow).reshape(())
    return t


def save(net, prefix: str, step: int, meta: Optional[dict] = None, loss_ema=None) -> str:
    """Saver.save(sess, prefix, global_step=step) with max_to_keep=1."""
    d = os.path.dirname(prefix)
    os.makedirs(d, exist_ok=True)
    base = os.path.basename(prefix)
    out = f"{prefix}-{step}"
    regularized = bool(meta and meta.get("regularization"))
    tf_bundle.write_bundle(out, to_tensors(net, loss_ema, regularized))
    for old in glob.glob(os.path.join(d, base + "-*")):
        if not old.startswith(out + "."):
            os.remove(old)
    with open(os.path.join(d, "checkpoint"), "w") as f:
        name = os.path.basename(out)
        f.write(f'model_checkpoint_path: "{name}"\nall_model_checkpoint_paths: "{name}"\n')
    return out


def latest_checkpoint(directory: str) -> Optional[str]:
    """tf.train.latest_checkpoint: the prefix the `checkpoint` file names
    (absolute, or relative to the directory -- the reference's Kaggle files hold
    absolute paths of another machine, README.md:84: fall back to the basename
    in this directory then)."""
    f = os.path.join(directory, "checkpoint")
    if os.path.exists(f):
        m = re.search(r'model_checkpoint_path: "([^"]+)"', open(f).read())
        if m:
            p = m.group(1)
            p = p if os.path.isabs(p) else os.path.join(directory, p)
            if _exists(p):
                return p
            local = os.path.join(directory, os.path.basename(p))
            if _exists(local):
                return local
    cands = sorted({re.search(r"(model-\d+)", x).group(1)
                    for x in glob.glob(os.path.join(directory, "model-*"))},
                   key=lambda s: int(s.split("-")[1]))
    return os.path.join(directory, cands[-1]) if cands else None


def _exists(prefix: str) -> bool:
    return os.path.exists(prefix + ".index") or os.path.exists(prefix + ".npz")


def restore(net, prefix: str) -> Optional[Tuple[float, int]]:
    """Saver.restore: parameters, Adam slots, beta powers, global_step.
    Returns the loss EMA state (shadow, 0) when the checkpoint has one."""
    if prefix.endswith(".npz") or (not os.path.exists(prefix + ".index")
                                   and os.path.exists(prefix + ".npz")):
        return _restore_npz(net, prefix)
    t = tf_bundle.read_bundle(prefix)
    n = net.n_params
    params, m, v = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for ours, tf, off, shape in tf_name_map(net.param_layout()):
        if tf not in t:
            raise ValueError(f"checkpoint {prefix} has no variable {tf} ({ours})")
        if tuple(t[tf].shape) != shape:
            raise ValueError(f"{tf}: checkpoint shape {t[tf].shape} != model shape {shape}")
        k = int(np.prod(shape))
        params[off:off + k] = t[tf].ravel()
        if tf + "/Adam" in t:
            m[off:off + k] = t[tf + "/Adam"].ravel()
            v[off:off + k] = t[tf + "/Adam_1"].ravel()
    net.set_params(params)
    net.set_optimizer_state(m, v, int(t.get("global_step", 0)),
                            float(t.get("beta1_power", 0.9)), float(t.get("beta2_power", 0.999)))
    for op in ("loss/add", "loss/add_1"):  # the total loss's EMA
        base = op + "/ExponentialMovingAverage"
        if base in t:
            return float(t[base]), 0
    return None


def _restore_npz(net, prefix: str):
    path = prefix if prefix.endswith(".npz") else prefix + ".npz"
    with np.load(path, allow_pickle=False) as z:
        names = [str(s) for s in z["names"]]
        if names != [n for n, _, _ in net.param_layout()]:
            raise ValueError(f"checkpoint {path} does not match the model's variables")
        net.set_params(z["params"])
        net.set_optimizer_state(z["adam_m"], z["adam_v"], int(z["global_step"]),
                                float(z["beta1_power"]), float(z["beta2_power"]))
    return None
