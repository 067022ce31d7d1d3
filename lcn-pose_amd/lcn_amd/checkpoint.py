"""Checkpoints in the reference's directory layout.

tf.compat.v1.train.Saver(max_to_keep=1) writes ``<dir>/model-<step>.*`` plus a
``checkpoint`` text file naming the latest prefix (models_att.py:161-162,
256-260, 321-322); tf.train.latest_checkpoint reads that file (:457-459).
This module keeps that layout; the payload is ``model-<step>.npz`` holding the
flat parameters (TF variable order, lcn_param_layout), both Adam slots,
global_step and the beta powers -- everything the reference checkpoint holds
for this model.
"""
from __future__ import annotations

import glob
import json
import os
import re
from typing import Optional

import numpy as np


def save(net, prefix: str, step: int, meta: Optional[dict] = None) -> str:
    d = os.path.dirname(prefix)
    os.makedirs(d, exist_ok=True)
    base = os.path.basename(prefix)
    params = net.get_params()
    m, v, gs, b1p, b2p = net.get_optimizer_state()
    layout = net.param_layout()
    out = f"{prefix}-{step}"
    tmp = out + ".tmp.npz"
    np.savez(tmp, params=params, adam_m=m, adam_v=v, global_step=np.int64(gs),
             beta1_power=np.float32(b1p), beta2_power=np.float32(b2p),
             names=np.array([n for n, _, _ in layout]),
             offsets=np.array([o for _, o, _ in layout], np.int64),
             meta=np.array(json.dumps(meta or {})))
    os.replace(tmp, out + ".npz")
    # max_to_keep=1
    for old in glob.glob(os.path.join(d, base + "-*")):
        if not old.startswith(out + "."):
            os.remove(old)
    with open(os.path.join(d, "checkpoint"), "w") as f:
        name = os.path.basename(out)
        f.write(f'model_checkpoint_path: "{name}"\nall_model_checkpoint_paths: "{name}"\n')
    return out


def latest_checkpoint(directory: str) -> Optional[str]:
    f = os.path.join(directory, "checkpoint")
    if os.path.exists(f):
        m = re.search(r'model_checkpoint_path: "([^"]+)"', open(f).read())
        if m:
            p = m.group(1)
            return p if os.path.isabs(p) else os.path.join(directory, p)
    cands = sorted(glob.glob(os.path.join(directory, "model-*.npz")),
                   key=lambda p: int(re.search(r"model-(\d+)", p).group(1)))
    return cands[-1][:-4] if cands else None


def restore(net, prefix: str) -> None:
    path = prefix if prefix.endswith(".npz") else prefix + ".npz"
    with np.load(path, allow_pickle=False) as z:
        names = [str(s) for s in z["names"]]
        layout = net.param_layout()
        if names != [n for n, _, _ in layout]:
            raise ValueError(f"checkpoint {path} does not match the model's variables")
        net.set_params(z["params"])
        net.set_optimizer_state(z["adam_m"], z["adam_v"], int(z["global_step"]),
                                float(z["beta1_power"]), float(z["beta2_power"]))
