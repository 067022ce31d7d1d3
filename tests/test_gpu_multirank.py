"""liblcn's data-parallel step with world 2 and 3, on one GPU.

RCCL refuses two ranks on one device, so the ranks here are liblcn handles
on the same GPU, one per Python thread, joined by a host-exchange
communicator (lcn_comm_init_host): every exchange of the multi-GPU step --
the ranks' row counts, the SyncBN sums of the forward and backward phases
(models_att.py:588-612 over the whole batch), the loss and the raw gradient
vector before Adam -- copies its device buffer to the host and is summed
across the threads.  Everything else is the code an RCCL run executes.

Checked against (a) one handle stepping the whole batch and (b) the float64
oracle: outputs, the loss, every gradient and two Adam steps, with equal,
uneven / ragged and three-way shards, the exponential mask with
regularisation, and dropout (the masks are keyed by the global row).
"""
import threading

import numpy as np
import pytest

import lcn_oracle as O
from lcn_testutil import make_cfg, make_network, perturbed_params, rel_err, synthetic_batch

pytestmark = pytest.mark.gpu


class ThreadAllReduce:
    """In-process all-reduce over `world` threads: sums (or maxes) the ranks'
    buffers in rank order in their own dtype, every rank gets the result."""

    def __init__(self, world, timeout=120.0):
        self.world = world
        self.barrier = threading.Barrier(world, timeout=timeout)
        self.bufs = [None] * world
        self.calls = [0] * world
        self.result = None

    def for_rank(self, rank):
        def allreduce(arr, op):
            self.calls[rank] += 1
            self.bufs[rank] = arr
            self.barrier.wait()
            if rank == 0:
                assert len({(b.size, b.dtype) for b in self.bufs}) == 1, "ranks disagree on the exchange"
                tot = self.bufs[0].copy()
                for b in self.bufs[1:]:
                    tot = np.maximum(tot, b) if op == "max" else tot + b
                self.result = tot
            self.barrier.wait()
            arr[:] = self.result
            self.barrier.wait()
        return allreduce


def run_ranks(world, fn):
    """fn(rank) on one thread per rank; returns the results by rank."""
    res, errs = [None] * world, []

    def body(r):
        try:
            res[r] = fn(r)
        except BaseException as e:  # noqa: BLE001
            errs.append((r, e))

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(600)
    assert not errs, errs
    return res


CASES = {
    "lc_knn3": dict(F=64, L=2, knn=3),
    "lc_knn1_nores": dict(F=64, L=1, knn=1, residual=False),
    "exp_reg": dict(F=64, L=1, mask="exponential", regularization=1e-3),
    # several 64-feature slabs per joint: the phased SyncBN finish folds the
    # slabs of a joint into channels (spj = 2 and 4)
    "lc_F128": dict(F=128, L=1, knn=2),
    "cfg4_shape": dict(F=256, L=2, knn=2, mask="exponential"),
}
# The wide cases are held to the one-handle run only (1e-5: their float32 sums
# are split differently); the one-handle path itself is checked against the
# float64 oracle at these shapes, with LeakyReLU kink handling, in
# tests/test_gpu_parity.py.
WIDE = {"lc_F128", "cfg4_shape"}


@pytest.mark.parametrize("case,sizes", [
    ("lc_knn3", [64, 64]),
    ("lc_knn3", [77, 45]),            # ragged 32-row tiles, uneven shards
    ("lc_knn1_nores", [40, 33, 55]),  # three ranks
    ("exp_reg", [96, 32]),
    ("lc_F128", [48, 48]),
    ("cfg4_shape", [48, 48]),
    ("cfg4_shape", [50, 46]),
], ids=["equal2", "ragged2", "three", "exp_reg", "F128", "cfg4_equal2", "cfg4_ragged2"])
def test_sharded_step_equals_full_batch(case, sizes):
    world, B = len(sizes), sum(sizes)
    cfg = make_cfg(**CASES[case])
    params = perturbed_params(cfg, seed=3)
    flat = O.flatten(cfg, params)
    x, lab = synthetic_batch(B, seed=11)
    x2, lab2 = synthetic_batch(B, seed=12)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    ar = ThreadAllReduce(world)

    def rank_fn(r):
        net = make_network(cfg, max_batch=max(sizes))
        net.comm_init_host(r, world, ar.for_rank(r))
        net.set_params(flat)
        sl = slice(offs[r], offs[r + 1])
        out, floss = net.forward_loss(x[sl], lab[sl])
        loss, _ = net.train_step(x[sl], lab[sl], update=False, keep_grads=True)
        grads = net.get_grads()
        # two Adam steps on two different global batches
        l1, _ = net.train_step(x[sl], lab[sl])
        l2, _ = net.train_step(x2[sl], lab2[sl])
        theta = net.get_params()
        net.close()
        return dict(out=out, floss=floss, loss=loss, grads=grads, l1=l1, l2=l2, theta=theta)

    res = run_ranks(world, rank_fn)

    # (a) one handle, whole batch
    one = make_network(cfg, max_batch=B)
    one.set_params(flat)
    out1, floss1 = one.forward_loss(x, lab)
    loss1, _ = one.train_step(x, lab, update=False, keep_grads=True)
    g1 = one.get_grads()
    l11, _ = one.train_step(x, lab)
    l12, _ = one.train_step(x2, lab2)
    theta1 = one.get_params()
    one.close()

    # (b) float64 oracle
    wide = case in WIDE
    tol = 1e-5 if wide else 1e-6
    out64, cache = O.forward(cfg, params, x, np.float64)
    loss64 = O.mse_loss(out64, lab) + O.reg_loss(cfg, params)
    g64 = None if wide else O.backward(cfg, params, cache, lab, np.float64)

    for r in range(world):
        sl = slice(offs[r], offs[r + 1])
        got = res[r]
        assert np.abs(got["out"] - out1[sl]).max() <= tol
        assert np.abs(got["out"] - out64[sl]).max() <= 1e-4
        # every rank reports the loss of the whole batch
        for k, ref in (("floss", floss1), ("loss", loss1), ("l1", l11), ("l2", l12)):
            assert abs(got[k] - ref) <= tol * max(1.0, abs(ref)), (k, got[k], ref)
        assert abs(got["loss"] - loss64) <= 1e-6 + 1e-5 * abs(loss64)
        # the all-reduced gradient, identical on every rank
        np.testing.assert_array_equal(got["grads"], res[0]["grads"])
        gr, g1u = O.unflatten(cfg, got["grads"]), O.unflatten(cfg, g1)
        for name, _ in O.param_specs(cfg):
            assert rel_err(gr[name], g1u[name]) <= tol, name
            if g64 is not None:
                assert rel_err(gr[name], g64[name]) <= 1e-4, name
        # two Adam steps: replicas stay identical and follow the one-handle run
        np.testing.assert_array_equal(got["theta"], res[0]["theta"])
        assert np.abs(got["theta"] - theta1).max() <= tol
    # the ranks made the same number of exchanges
    assert len(set(ar.calls)) == 1


@pytest.mark.parametrize("L", [0, 1, 3])
def test_collectives_per_step(L):
    """A data-parallel training step makes 4L + 3 exchanges: one SyncBN
    all-reduce per BN layer forward (1 + 2L; layer 0's also carries the ranks'
    batch rows) and backward (1 + 2L; the first also carries the loss sum), and
    one of the raw gradient vector.  forward_loss: 1 + 2L and the loss."""
    sizes, world = [40, 56], 2
    cfg = make_cfg(F=64, L=L, knn=2)
    flat = O.flatten(cfg, perturbed_params(cfg, seed=4))
    x, lab = synthetic_batch(sum(sizes), seed=9)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    ar = ThreadAllReduce(world)

    def rank_fn(r):
        net = make_network(cfg, max_batch=max(sizes))
        net.comm_init_host(r, world, ar.for_rank(r))
        net.set_params(flat)
        sl = slice(offs[r], offs[r + 1])
        assert net.comm_info() == ("host", r, world)
        c0 = ar.calls[r]
        loss, _ = net.train_step(x[sl], lab[sl])
        c1 = ar.calls[r]
        net.forward_loss(x[sl], lab[sl])
        c2 = ar.calls[r]
        net.forward(x[sl])
        c3 = ar.calls[r]
        net.close()
        return c1 - c0, c2 - c1, c3 - c2, loss

    res = run_ranks(world, rank_fn)
    for step_calls, floss_calls, fwd_calls, _ in res:
        assert step_calls == 4 * L + 3
        assert floss_calls == 2 * L + 2
        assert fwd_calls == 2 * L + 1
    assert res[0][3] == res[1][3]


def test_suspended_calls_make_no_exchange_with_phased_reductions(monkeypatch):
    """With the phased (multi-GPU) BN reductions forced on, a suspended
    communicator keeps every exchange off: ranks predict different numbers of
    batches rank-locally (no deadlock, no all-reduce call) and get the
    one-handle results."""
    monkeypatch.setenv("LCN_FORCE_PHASED", "1")
    world, bs = 2, 32
    cfg = make_cfg(F=64, L=1, knn=2)
    flat = O.flatten(cfg, perturbed_params(cfg, seed=6))
    x, _ = synthetic_batch(3 * bs, seed=8)
    rows = [x[:2 * bs], x[2 * bs:]]       # two batches on rank 0, one on rank 1
    ar = ThreadAllReduce(world)

    def rank_fn(r):
        net = make_network(cfg, max_batch=bs)
        net.comm_init_host(r, world, ar.for_rank(r))
        net.set_params(flat)
        net.comm_suspend(True)
        c0 = ar.calls[r]
        net.dataset_upload(0, rows[r].astype(np.float64))
        p = net.predict_dataset(0, rows[r].shape[0], bs)
        calls = ar.calls[r] - c0
        net.comm_suspend(False)
        net.close()
        return p, calls

    res = run_ranks(world, rank_fn)
    monkeypatch.delenv("LCN_FORCE_PHASED")
    one = make_network(cfg, max_batch=bs)
    one.set_params(flat)
    for r in range(world):
        assert res[r][1] == 0
        one.dataset_upload(0, rows[r].astype(np.float64))
        ref = one.predict_dataset(0, rows[r].shape[0], bs)
        assert np.abs(res[r][0] - ref).max() <= 1e-6
    one.close()


def test_dropout_masks_follow_the_global_row():
    """tf.nn.dropout's mask is keyed by the global row, so shards [40, 88]
    draw the masks of the whole 128-row batch (lcn_internal.h Dropout)."""
    sizes, world = [40, 88], 2
    B = sum(sizes)
    cfg = make_cfg(F=64, L=1, knn=2)
    params = perturbed_params(cfg, seed=5)
    flat = O.flatten(cfg, params)
    x, lab = synthetic_batch(B, seed=21)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    ar = ThreadAllReduce(world)

    def rank_fn(r):
        net = make_network(cfg, max_batch=max(sizes))
        net.comm_init_host(r, world, ar.for_rank(r))
        net.set_params(flat)
        net.set_dropout(0.3, seed=77)
        sl = slice(offs[r], offs[r + 1])
        loss, _ = net.train_step(x[sl], lab[sl], update=False, keep_grads=True)
        g = net.get_grads()
        net.close()
        return loss, g

    res = run_ranks(world, rank_fn)
    one = make_network(cfg, max_batch=B)
    one.set_params(flat)
    one.set_dropout(0.3, seed=77)
    loss1, _ = one.train_step(x, lab, update=False, keep_grads=True)
    g1 = O.unflatten(cfg, one.get_grads())
    one.close()
    for loss, g in res:
        assert abs(loss - loss1) <= 1e-6 * max(1.0, abs(loss1))
        gu = O.unflatten(cfg, g)
        for name, _ in O.param_specs(cfg):
            assert rel_err(gu[name], g1[name]) <= 2e-6, name


def test_predict_dataset_shards_form_one_syncbn_batch():
    """lcn_predict_dataset with two ranks: rank r's batch i and the other
    rank's batch i are one BN batch; with the dataset split at a batch
    boundary the predictions equal one handle predicting with 2x the batch."""
    bs, world = 48, 2
    cfg = make_cfg(F=64, L=1, knn=3)
    params = perturbed_params(cfg, seed=2)
    flat = O.flatten(cfg, params)
    x, _ = synthetic_batch(2 * bs, seed=4)
    ar = ThreadAllReduce(world)

    def rank_fn(r):
        net = make_network(cfg, max_batch=bs)
        net.comm_init_host(r, world, ar.for_rank(r))
        net.set_params(flat)
        net.dataset_upload(0, x[r * bs:(r + 1) * bs].astype(np.float64))
        p = net.predict_dataset(0, bs, bs)
        net.close()
        return p

    res = run_ranks(world, rank_fn)
    one = make_network(cfg, max_batch=2 * bs)
    one.set_params(flat)
    one.dataset_upload(0, x.astype(np.float64))
    ref = one.predict_dataset(0, 2 * bs, 2 * bs)
    one.close()
    got = np.concatenate(res, axis=0)
    assert np.abs(got - ref).max() <= 1e-6


def test_failing_exchange_is_reported_not_hung():
    """An exception in the caller's all-reduce surfaces as LCN_E_COMM."""
    from lcn_amd.native import LcnNativeError
    cfg = make_cfg(F=64, L=1, knn=1)
    net = make_network(cfg, max_batch=32)

    def boom(arr, op):
        raise RuntimeError("transport down")

    net.comm_init_host(0, 1, boom)
    net.set_params(O.flatten(cfg, perturbed_params(cfg, seed=1)))
    x, lab = synthetic_batch(32, seed=0)
    with pytest.raises(LcnNativeError, match="all-reduce"):
        net.train_step(x, lab)
    with pytest.raises(LcnNativeError):  # one communicator per handle
        net.comm_init_host(0, 1, boom)
    net.close()
