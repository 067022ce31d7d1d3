"""Data-parallel decomposition (world > 1) on CPU over gloo.

liblcn runs a multi-GPU step as: per-rank 128-row tile moments of every BN
layer -> RCCL all-reduce (float64) -> SyncBN statistics; per-rank BN-backward
sums -> all-reduce -> dz coefficients; LOCAL raw gradients (dW_e, db, dgamma,
dbeta with the global-batch loss scale) -> one all-reduce of the raw-gradient
vector -> mask / clip backward, regularisation and Adam on every rank
(lcn-pose_amd/csrc/lcn_api.cpp bn_stats, bn_back, finish_device).

oracle.sharded_grads restates exactly that decomposition; these tests run it on
2 and 3 gloo ranks with uneven, ragged shards and check it reproduces the
single-process full-batch oracle (models_att.py:588-612 with the whole batch)
to float64 round-off.  The GPU kernels implement the same per-rank pieces
(tests/test_gpu_parity.py checks those against the oracle on one GPU).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import lcn_oracle as O
from lcn_testutil import make_cfg, perturbed_params, synthetic_batch


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


CASES = {
    "lc_knn3": dict(F=64, L=2, knn=3),
    "lc_knn1_nores": dict(F=64, L=1, knn=1, residual=False),
    "exp_reg": dict(F=64, L=1, mask="exponential", regularization=1e-3),
}


def _worker(rank, world, port, case, sizes, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kw = dict(CASES[case])
        cfg = make_cfg(**kw)
        params = perturbed_params(cfg, seed=3)
        x, lab = synthetic_batch(sum(sizes), seed=11)
        r0 = sum(sizes[:rank])
        xs, ls = x[r0:r0 + sizes[rank]], lab[r0:r0 + sizes[rank]]

        def allreduce(a):
            t = torch.tensor(np.asarray(a, np.float64))  # a copy: the caller's array stays local
            dist.all_reduce(t)
            return t.numpy()

        out, g = O.sharded_grads(cfg, params, xs, ls, allreduce, world)
        q.put((rank, out, {k: np.asarray(v) for k, v in g.items()}))
    finally:
        dist.destroy_process_group()


def _run(case, sizes):
    world = len(sizes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, out, g = q.get(timeout=300)
        res[rank] = (out, g)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("case,sizes", [
    ("lc_knn3", [64, 64]),
    ("lc_knn3", [77, 45]),           # ragged 32-row tiles, uneven shards
    ("lc_knn1_nores", [40, 33, 55]),  # three ranks
    ("exp_reg", [96, 32]),
])
def test_sharded_step_equals_full_batch(case, sizes):
    res = _run(case, sizes)
    cfg = make_cfg(**CASES[case])
    params = perturbed_params(cfg, seed=3)
    x, lab = synthetic_batch(sum(sizes), seed=11)
    out_ref, cache = O.forward(cfg, params, x, dtype=np.float64)
    g_ref = O.backward(cfg, params, cache, lab, dtype=np.float64)
    # every rank ends with the same global gradient
    for r in range(len(sizes)):
        out, g = res[r]
        r0 = sum(sizes[:r])
        np.testing.assert_allclose(out, out_ref[r0:r0 + sizes[r]], rtol=1e-10, atol=1e-12)
        assert set(g) == set(g_ref)
        for k in g_ref:
            np.testing.assert_allclose(g[k], g_ref[k], rtol=1e-9, atol=1e-12, err_msg=k)


def test_sharded_single_rank_is_full_batch():
    cfg = make_cfg(F=64, L=1, knn=2)
    params = perturbed_params(cfg, seed=5)
    x, lab = synthetic_batch(70, seed=2)
    out, g = O.sharded_grads(cfg, params, x, lab, lambda a: np.asarray(a, np.float64), 1)
    out_ref, cache = O.forward(cfg, params, x, dtype=np.float64)
    g_ref = O.backward(cfg, params, cache, lab, dtype=np.float64)
    np.testing.assert_allclose(out, out_ref, rtol=1e-12, atol=1e-12)
    for k in g_ref:
        np.testing.assert_allclose(g[k], g_ref[k], rtol=1e-10, atol=1e-13, err_msg=k)
