"""Parameter initialisation of the product path (host side).

cgcnn.kaiming (models_att.py:614-628): truncated_normal(stddev=1, +-2 sigma)
* sqrt(2 / shape[0]) for every weight and bias (biases: shape[0] = len(b));
the LC mask variable starts at L = N^T (init_type 'same', :549-566); Keras
BatchNormalization gamma = 1, beta = 0.  TF's RNG is unseeded in the
reference, so only the distribution is reproduced.
"""
from __future__ import annotations

import math
from typing import Iterable, Tuple

import numpy as np


def truncated_normal(rng: np.random.Generator, shape) -> np.ndarray:
    out = rng.standard_normal(size=shape)
    bad = np.abs(out) > 2.0
    while bad.any():
        out[bad] = rng.standard_normal(size=int(bad.sum()))
        bad = np.abs(out) > 2.0
    return out


def init_flat(layout: Iterable[Tuple[str, int, tuple]], n_params: int, neighbour: np.ndarray,
              seed=None) -> np.ndarray:
    """Flat float32 parameter vector in the C-ABI layout (lcn_param_layout)."""
    rng = np.random.default_rng(seed)
    flat = np.empty(n_params, np.float32)
    for name, off, shape in layout:
        n = int(np.prod(shape))
        if name == "mask":
            v = np.asarray(neighbour, np.float32).T
        elif name.endswith("_gamma"):
            v = np.ones(shape, np.float32)
        elif name.endswith("_beta"):
            v = np.zeros(shape, np.float32)
        else:
            v = truncated_normal(rng, shape) * math.sqrt(2.0 / shape[0])
        flat[off:off + n] = np.asarray(v, np.float32).ravel()
    return flat
