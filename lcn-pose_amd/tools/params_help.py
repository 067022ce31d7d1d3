"""Hyper-parameter dictionary and LCN structure matrix for cgcnn(**params).

Behaviour follows the reference's tools/params_help.py:
  get_neighbour_matrix_by_hand  :8-20   (N = 1[(A + I)^knn != 0])
  update_parameters             :92-119 (CLI overrides, in that order)
  get_params                    :122-173 (defaults)
"""
from __future__ import annotations

import numpy as np

try:
    from . import filter_hub
except ImportError:  # imported as a top-level module (sys.path = tools/)
    import filter_hub  # type: ignore

N_JOINTS = 17


def get_neighbour_matrix_by_hand(neighbour_dict, knn=1):
    """Self-loops plus skeleton edges, expanded to the knn-hop neighbourhood."""
    if len(neighbour_dict) != N_JOINTS:
        raise AssertionError("the LCN is built for 17 joints")
    adj = np.eye(N_JOINTS, dtype=np.float32)
    for joint, nbrs in neighbour_dict.items():
        adj[joint, nbrs] = 1.0
    if knn < 2:
        return adj
    reach = np.linalg.matrix_power(adj, knn)
    return (reach != 0).astype(np.float32)


_DEFAULTS = dict(
    dir_name="test1/", num_epochs=200, batch_size=200, decay_type="exp",
    F=64, mask_type="locally_connected", init_type="random",
    in_joints=N_JOINTS, out_joints=N_JOINTS, num_layers=3, in_F=2,
    residual=True, max_norm=True, batch_norm=True, regularization=0,
    learning_rate=1e-3, checkpoints="final", knn=1,
)


def get_params(is_training, gt_dataset=None):
    """Default parameter dictionary (gt_dataset is unused, as in the reference)."""
    params = dict(_DEFAULTS)
    params["decay_params"] = {"decay_steps": 32000, "decay_rate": 0.96}
    params["neighbour_matrix"] = get_neighbour_matrix_by_hand(filter_hub.neighbour_dict_set[0], knn=1)
    params["dropout"] = 0.25 if is_training else 0
    params["is_training"] = is_training
    return params


def update_parameters(args, params):
    """Apply command-line overrides (truthiness rules of the reference)."""
    if args.test_indices:
        params["dir_name"] = "test" + args.test_indices + "/"
    if args.knn:
        params["knn"] = args.knn
        params["neighbour_matrix"] = get_neighbour_matrix_by_hand(filter_hub.neighbour_dict_set[0],
                                                                  knn=args.knn)
    if args.layers is not None:
        params["num_layers"] = args.layers
    if args.dropout is not None:
        params["dropout"] = args.dropout
    if getattr(args, "channels", None):
        params["F"] = args.channels
    if getattr(args, "checkpoints", None):
        params["checkpoints"] = args.checkpoints
    for key, attr in (("mask_type", "mask_type"), ("init_type", "init_type"),
                      ("num_epochs", "epochs"), ("batch_size", "batch_size")):
        value = getattr(args, attr)
        if value:
            params[key] = value
    for key in ("learning_rate", "regularization"):
        if hasattr(args, key):
            params[key] = getattr(args, key)
