"""HIP path vs the CPU oracle (runs on the MI355X box: pytest -m gpu).

Tolerances: forward outputs |d| <= 1e-4 in
normalised units against the float64 oracle; gradients <= 1e-4 relative
(per tensor, L2) against float64; one Adam step |d theta| <= 1e-6 absolute.
"""
import numpy as np
import pytest

import lcn_oracle as O
from lcn_testutil import make_cfg, make_network, perturbed_params, rel_err, synthetic_batch

pytestmark = pytest.mark.gpu

CASES = [
    # name, cfg kwargs, B
    ("lc_knn3_L3", dict(F=64, L=3, knn=3), 256),
    ("lc_knn3_B200", dict(F=64, L=3, knn=3), 200),
    ("lc_knn1_L2", dict(F=64, L=2, knn=1), 128),
    ("lc_knn2_L3", dict(F=64, L=3, knn=2), 300),
    ("lc_knn5_L1", dict(F=64, L=1, knn=5), 64),
    ("exp_L2_F128", dict(F=128, L=2, knn=2, mask="exponential"), 96),
    # four slabs per joint, every joint pair: 68 blocks an output slab, the weight
    # gradient in groups of four blocks (gemm_dw4.hip)
    ("exp_L1_F256", dict(F=256, L=1, knn=2, mask="exponential"), 64),
    # three slabs per joint: two pair up, the third finds its partner across joints
    ("lc_F192_knn4", dict(F=192, L=1, knn=4), 70),
    ("lc_inF3", dict(F=64, L=1, knn=3, in_F=3), 160),
    ("lc_nores", dict(F=64, L=2, knn=3, residual=False), 128),
    ("lc_nobn", dict(F=64, L=1, knn=2, batch_norm=False), 128),
    ("lc_noclip_reg", dict(F=64, L=1, knn=2, max_norm=False, regularization=0.01), 64),
    ("lc_tiny_B7", dict(F=64, L=1, knn=3), 7),
    # 80 row tiles: the largest batch of the small-batch GEMM; 81: the first of the other
    ("lc_B2560", dict(F=64, L=1, knn=2), 2560),
    ("lc_B2570", dict(F=64, L=1, knn=2), 2570),
    # BASELINE.json configs[4] (cfg5) model shape: knn 5, 3 blocks
    ("cfg5_knn5_L3", dict(F=64, L=3, knn=5), 512),
]


# Batches of up to 2560 rows run the small-batch GEMM kernel (gemm_small.hip);
# LCN_SMALL_RT=0 at handle creation keeps such a batch on the large-batch
# kernels: one output slab per workgroup (gemm_bs.hip, LCN_GEMM_PAIR=0) or two
# (gemm_pair.hip, LCN_GEMM_PAIR=1), so all three are held to the oracle on the
# same cases.
@pytest.fixture(params=["small_batch_gemm", "large_batch_gemm", "paired_slab_gemm"])
def gemm_path(request, monkeypatch):
    if request.param != "small_batch_gemm":
        monkeypatch.setenv("LCN_SMALL_RT", "0")
        monkeypatch.setenv("LCN_GEMM_PAIR", "1" if request.param == "paired_slab_gemm" else "0")
    return request.param


def _setup(kw, B, seed=0):
    cfg = make_cfg(**kw)
    params = perturbed_params(cfg, seed=1 + seed)
    x, lab = synthetic_batch(B, cfg.in_F, seed=seed)
    net = make_network(cfg, max_batch=max(B, 8))
    net.set_params(O.flatten(cfg, params))
    return cfg, params, x, lab, net


@pytest.mark.parametrize("name,kw,B", CASES, ids=[c[0] for c in CASES])
def test_forward_matches_oracle(name, kw, B, gemm_path):
    cfg, params, x, lab, net = _setup(kw, B)
    out = net.forward(x)
    ref64, _ = O.forward(cfg, params, x, np.float64)
    err = np.abs(out - ref64).max()
    assert err <= 1e-4, f"max |out - oracle64| = {err}"
    out2, loss = net.forward_loss(x, lab)
    np.testing.assert_array_equal(out, out2)
    # op_loss = mse + reg * sum l2_loss(W, b)  (models_att.py:356-365)
    expect = O.mse_loss(ref64, lab) + O.reg_loss(cfg, params)
    assert abs(loss - expect) <= 1e-6 + 1e-5 * abs(expect)


@pytest.mark.parametrize("name,kw,B", CASES, ids=[c[0] for c in CASES])
def test_gradients_match_oracle(name, kw, B, gemm_path):
    cfg, params, x, lab, net = _setup(kw, B)
    loss, lr = net.train_step(x, lab, update=False, keep_grads=True)
    g = O.unflatten(cfg, net.get_grads())
    out64, cache = O.forward(cfg, params, x, np.float64)
    ref = O.backward(cfg, params, cache, lab, np.float64)
    expect = O.mse_loss(out64, lab) + O.reg_loss(cfg, params)
    assert abs(loss - expect) <= 1e-6 + 1e-5 * abs(expect)
    # tolerance: 1e-4 relative, or twice the float32 restatement's own
    # deviation from float64 where the case is that ill-conditioned
    # (small batch + dense mask: BN-parameter sums cancel)
    out32, cache32 = O.forward(cfg, params, x, np.float32)
    ref32 = O.backward(cfg, params, cache32, lab, np.float32)
    bad = {}
    for name_, _ in O.param_specs(cfg):
        e = rel_err(g[name_], ref[name_])
        tol = max(1e-4, 2.0 * rel_err(ref32[name_], ref[name_]))
        if e > tol:
            bad[name_] = (e, tol)
    assert not bad, f"relative gradient errors above 1e-4: {bad}"
    # params unchanged without update
    np.testing.assert_array_equal(net.get_params(), O.flatten(cfg, params))


def test_weight_gradient_in_pairs_of_blocks_at_four_slabs_per_joint(monkeypatch):
    """LCN_DW_QUAD=0 keeps the two-block weight-gradient kernel where the
    four-block one would run (every output slab a multiple of four blocks):
    the same gradients."""
    monkeypatch.setenv("LCN_DW_QUAD", "0")
    test_gradients_match_oracle("exp_L1_F256", dict(F=256, L=1, knn=2, mask="exponential"), 64, "default")


def test_adam_step_matches_oracle(gemm_path):
    cfg, params, x, lab, net = _setup(dict(F=64, L=2, knn=3), 256)
    st = O.adam_init(cfg, params)
    p_ref = {k: v.copy() for k, v in params.items()}
    for step in range(3):
        xs, ls = synthetic_batch(256, 2, seed=10 + step)
        _, lr = net.train_step(xs, ls)
        out64, cache = O.forward(cfg, p_ref, xs, np.float64)
        g = O.backward(cfg, p_ref, cache, ls, np.float64)
        lr_ref = O.adam_step(cfg, p_ref, {k: v.astype(np.float32) for k, v in g.items()}, st)
        assert lr == pytest.approx(float(lr_ref), rel=1e-6)
    got = O.unflatten(cfg, net.get_params())
    for k in p_ref:
        d = np.abs(got[k] - p_ref[k]).max()
        assert d <= 5e-6, (k, d)
    m, v, gs, b1p, b2p = net.get_optimizer_state()
    assert gs == 3 and b1p == pytest.approx(0.9 ** 4, rel=1e-6)


def test_train_loss_decreases():
    cfg, params, x, lab, net = _setup(dict(F=64, L=3, knn=3), 512)
    losses = [net.train_step(x, lab)[0] for _ in range(30)]
    assert losses[-1] < 0.8 * losses[0], losses
    assert all(b < a for a, b in zip(losses, losses[1:])), losses


def test_duplicated_batch_gives_same_gradients():
    """Size-independent property: BN statistics and mean-loss gradients are
    invariant to duplicating every pose (checks the batch reductions at
    large B without running the oracle there)."""
    cfg = make_cfg(F=64, L=3, knn=3)
    params = perturbed_params(cfg)
    x, lab = synthetic_batch(8192, 2, seed=3)
    net = make_network(cfg, max_batch=16384)
    net.set_params(O.flatten(cfg, params))
    net.train_step(x, lab, update=False, keep_grads=True)
    g1 = net.get_grads()
    net.train_step(np.concatenate([x, x]), np.concatenate([lab, lab]), update=False,
                   keep_grads=True)
    g2 = net.get_grads()
    for name, off, shape in net.param_layout():
        n = int(np.prod(shape))
        assert rel_err(g2[off:off + n], g1[off:off + n]) < 1e-4, name


@pytest.mark.parametrize("kw,B", [(dict(F=64, L=2, knn=3), 8192 + 40),
                                  (dict(F=256, L=1, knn=2, mask="exponential"), 2624)],
                         ids=["lc_F64", "exp_F256"])
def test_training_steps_are_bitwise_reproducible(kw, B):
    """The same three training steps on two handles: losses, gradients and the
    updated parameters agree bit for bit.  Nothing in a step depends on the
    order in which workgroups finish: the batch statistics are summed in a
    fixed order (the workgroup that finishes the column sums last only runs
    the per-channel finish), every weight-gradient partial has one writer and
    the partials are added in slot order, the stored dz has one writer per
    item.  Batches of the large-batch kernels (one and two output slabs per
    workgroup, two and four blocks per weight-gradient workgroup)."""
    cfg = make_cfg(**kw)
    params = O.flatten(cfg, perturbed_params(cfg))
    runs = []
    for _ in range(2):
        net = make_network(cfg, max_batch=B)
        net.set_params(params)
        losses, grads = [], None
        for step in range(3):
            x, lab = synthetic_batch(B, cfg.in_F, seed=20 + step)
            loss, _ = net.train_step(x, lab, keep_grads=True)
            losses.append(loss)
            grads = net.get_grads().copy()
        runs.append((np.array(losses), grads, net.get_params().copy()))
        net.close()
    for a, b in zip(runs[0], runs[1]):
        np.testing.assert_array_equal(a, b)


def test_duplicated_batch_gives_same_gradients_cfg4_shape():
    """The same property at BASELINE.json configs[3]'s model shape (dense
    exponential mask, F 256, 6 blocks, H 4352) and its per-GPU batch on 8
    GPUs: 8 192 poses -> 16 384.  BN-parameter gradients at this shape are
    sums with heavy cancellation, hence the looser bar for them; a wrong
    batch reduction (a dropped tile, a wrong count) is off by far more."""
    cfg = make_cfg(F=256, L=6, knn=2, mask="exponential")
    params = perturbed_params(cfg)
    x, lab = synthetic_batch(8192, 2, seed=5)
    net = make_network(cfg, max_batch=16384)
    net.set_params(O.flatten(cfg, params))
    l1, _ = net.train_step(x, lab, update=False, keep_grads=True)
    g1 = net.get_grads()
    l2, _ = net.train_step(np.concatenate([x, x]), np.concatenate([lab, lab]), update=False,
                           keep_grads=True)
    g2 = net.get_grads()
    assert l2 == pytest.approx(l1, rel=1e-6)
    for name, off, shape in net.param_layout():
        n = int(np.prod(shape))
        tol = 1e-3 if name.endswith(("_gamma", "_beta")) else 1e-4
        assert rel_err(g2[off:off + n], g1[off:off + n]) < tol, name
    net.close()


def test_phased_reductions_match_single_pass(monkeypatch):
    """The multi-GPU reduction path (per-rank phase-1 sums -> all-reduce ->
    phase-2 finish, lcn_api.cpp bn_stats / bn_back) forced on one GPU, where
    the all-reduce is the identity, must reproduce the single-pass path."""
    cfg, params, x, lab, net = _setup(dict(F=64, L=2, knn=3), 300)
    loss0, _ = net.train_step(x, lab, update=False, keep_grads=True)
    g0 = net.get_grads()
    out0 = net.forward(x)
    monkeypatch.setenv("LCN_FORCE_PHASED", "1")
    net2 = make_network(cfg, max_batch=300)
    net2.set_params(O.flatten(cfg, params))
    loss1, _ = net2.train_step(x, lab, update=False, keep_grads=True)
    g1 = net2.get_grads()
    np.testing.assert_allclose(net2.forward(x), out0, rtol=0, atol=1e-6)
    assert loss1 == pytest.approx(loss0, rel=1e-6)
    for name, off, shape in net.param_layout():
        n = int(np.prod(shape))
        assert rel_err(g1[off:off + n], g0[off:off + n]) < 1e-6, name


def test_single_rank_rccl_communicator_runs_the_multi_gpu_path(monkeypatch):
    """lcn_comm_init with world 1 creates a real RCCL communicator, so every
    data-parallel exchange of the multi-GPU path runs on one GPU: the phased
    SyncBN reductions with their ncclAllReduce (float64), the gradient
    all-reduce (float32) before Adam and the loss all-reduce, plus the host
    all-reduce bench.py uses as a barrier.  A sum over one rank is the
    identity, so two Adam steps and a forward must equal, bit for bit, the
    same steps on the phased path without a communicator."""
    from lcn_amd.native import LcnNativeError, Network
    cfg, params, x, lab, net = _setup(dict(F=64, L=2, knn=3), 300)
    monkeypatch.setenv("LCN_FORCE_PHASED", "1")
    ref = make_network(cfg, max_batch=300)
    monkeypatch.delenv("LCN_FORCE_PHASED")
    ref.set_params(O.flatten(cfg, params))
    net.comm_init(Network.comm_unique_id(), 0, 1)
    losses = []
    for n in (ref, net):
        l1, _ = n.train_step(x, lab)
        l2, _ = n.train_step(x[::-1].copy(), lab[::-1].copy())
        losses.append((l1, l2))
    assert losses[0] == losses[1]
    assert np.array_equal(net.get_params(), ref.get_params())
    assert np.array_equal(net.forward(x), ref.forward(x))
    assert list(net.allreduce_host([1.5, -2.0])) == [1.5, -2.0]
    assert list(net.allreduce_host([3.0], op="max")) == [3.0]
    with pytest.raises(LcnNativeError):
        net.comm_init(Network.comm_unique_id(), 0, 1)


def test_full_size_cfg3_matches_oracle():
    """BASELINE.json configs[1] at its full size (B = 65 536, F = 64, L = 3,
    knn = 3): outputs and every gradient against the float64 oracle."""
    B = 65536
    cfg, params, x, lab, net = _setup(dict(F=64, L=3, knn=3), B, seed=4)
    out = net.forward(x)
    loss, _ = net.train_step(x, lab, update=False, keep_grads=True)
    g = O.unflatten(cfg, net.get_grads())
    out64, cache = O.forward(cfg, params, x, np.float64)
    assert np.abs(out - out64).max() <= 1e-4
    assert abs(loss - (O.mse_loss(out64, lab) + O.reg_loss(cfg, params))) <= 1e-5 * abs(loss)
    ref = O.backward(cfg, params, cache, lab, np.float64)
    del cache
    bad = {k: rel_err(g[k], ref[k]) for k, _ in O.param_specs(cfg) if rel_err(g[k], ref[k]) > 1e-4}
    assert not bad, bad


def _device_kinks(cfg, params, net, B):
    """LeakyReLU branch masks u > 0 of the device's own float32 forward (z and
    BN statistics of every BN layer through lcn_debug_tensor)."""
    H, F = 17 * cfg.F, cfg.F
    kinks = {}
    for k, (wn, bname, bnp, fin, fout) in enumerate(O.layer_names(cfg)):
        if bnp is None:
            continue
        z = net.debug_tensor(0, k, B * H).reshape(B, 17, F).astype(np.float64)
        st = net.debug_tensor(2, k, 2 * F)
        mean, rstd = st[:F].astype(np.float64), st[F:].astype(np.float64)
        u = (z - mean) * (rstd * params[bnp + "_gamma"]) + params[bnp + "_beta"]
        kinks[k] = (u > 0).reshape(B, H)
    return kinks


def test_cfg4_shape_matches_oracle():
    """BASELINE.json configs[3] (cfg4) model shape -- exponential (dense) mask,
    knn 2, 6 blocks, 256 channels (H = 4352, 227.7 M parameters) -- at a batch
    the float64 oracle finishes in seconds: outputs and every gradient.

    At this depth and width a few pre-activations u land within float32
    rounding of LeakyReLU's kink (|u| ~ 1e-6), and the float32 device forward
    then takes the other branch (slope 1 vs 0.2) than the float64 oracle:
    one such element moves a small-batch BN-parameter gradient by ~1e-3
    relative.  The gradients are therefore checked against the float64
    oracle differentiated at the device's own branches (oracle ``kinks``
    hook), and the branch disagreements are checked to be exactly those
    vanishing-|u| elements."""
    B = 96
    cfg, params, x, lab, net = _setup(dict(F=256, L=6, knn=2, mask="exponential"), B, seed=5)
    out = net.forward(x)
    loss, _ = net.train_step(x, lab, update=False, keep_grads=True)
    g = O.unflatten(cfg, net.get_grads())
    kinks = _device_kinks(cfg, params, net, B)
    out64, cache = O.forward(cfg, params, x, np.float64)
    assert np.abs(out - out64).max() <= 1e-4
    assert abs(loss - O.mse_loss(out64, lab)) <= 1e-5 * abs(loss)
    flips = 0
    for k, pos in kinks.items():
        u = cache["layers"][k]["u"]
        d = pos != (u > 0)
        flips += int(d.sum())
        if d.any():  # only where u is float32 rounding away from 0
            assert np.abs(u[d]).max() <= 1e-4 * np.sqrt(np.mean(u * u)), (k, np.abs(u[d]).max())
    assert flips <= 1e-5 * B * 17 * cfg.F * len(kinks), flips
    ref = O.backward(cfg, params, cache, lab, np.float64, kinks=kinks)
    del cache
    bad = {k: rel_err(g[k], ref[k]) for k, _ in O.param_specs(cfg) if rel_err(g[k], ref[k]) > 1e-4}
    print(f"kink branch disagreements: {flips}")
    assert not bad, bad


@pytest.mark.parametrize("L,B,rate,pair", [(3, 256, 0.3, "0"), (1, 200, 0.25, "0"), (2, 256, 0.3, "1")])
def test_dropout_training_step_matches_oracle(L, B, rate, pair, monkeypatch):
    """tf.nn.dropout after every BN + LeakyReLU (models_att.py:673, 700, 742)
    with the counter-based masks (oracle.dropout_mask): loss and every
    gradient of two consecutive training steps (mask step 0, then 1) against
    the float64 oracle; predict is unaffected by the dropout setting.  A step
    with dropout always takes a large-batch GEMM kernel: one output slab per
    workgroup, or two (pair)."""
    monkeypatch.setenv("LCN_GEMM_PAIR", pair)
    cfg, params, x, lab, net = _setup(dict(F=64, L=L, knn=3), B)
    seed = 0x1234_5678_9ABC
    net.set_dropout(rate, seed)
    for step in range(2):
        loss, _ = net.train_step(x, lab, update=False, keep_grads=True)
        g = O.unflatten(cfg, net.get_grads())
        kinks = _device_kinks(cfg, params, net, B)  # see test_cfg4_shape_matches_oracle
        out64, cache = O.forward(cfg, params, x, np.float64, drop=(rate, seed, step))
        assert abs(loss - O.mse_loss(out64, lab)) <= 1e-5 * abs(loss)
        for k, pos in kinks.items():
            u = cache["layers"][k]["u"]
            d = pos != (u > 0)
            assert d.sum() <= 2 and (not d.any() or np.abs(u[d]).max() <= 1e-4 * np.sqrt(np.mean(u * u)))
        ref = O.backward(cfg, params, cache, lab, np.float64, kinks=kinks)
        out32, c32 = O.forward(cfg, params, x, np.float32, drop=(rate, seed, step))
        ref32 = O.backward(cfg, params, c32, lab, np.float32, kinks=kinks)
        bad = {}
        for k, _ in O.param_specs(cfg):
            e, tol = rel_err(g[k], ref[k]), max(1e-4, 2.0 * rel_err(ref32[k], ref[k]))
            if e > tol:
                bad[k] = (e, tol)
        assert not bad, (step, bad)
    ref_plain, _ = O.forward(cfg, params, x, np.float64)
    assert np.abs(net.forward(x) - ref_plain).max() <= 1e-4
    net.set_dropout(0.0)
    loss0, _ = net.train_step(x, lab, update=False)
    assert abs(loss0 - O.mse_loss(ref_plain, lab)) <= 1e-5 * abs(loss0)


def test_step_graphs_replay_the_direct_launches(monkeypatch):
    """Training steps replayed from a captured HIP graph (world 1, no dropout)
    give bit-identical losses, parameters and optimiser state to the same
    steps launched kernel by kernel (LCN_GRAPHS=0), across batch sizes,
    update / no-update and keep-grads variants."""
    cfg = make_cfg(F=64, L=2, knn=3)
    params = perturbed_params(cfg, seed=2)
    nets = []
    for g in ("1", "0"):
        monkeypatch.setenv("LCN_GRAPHS", g)
        n = make_network(cfg, max_batch=512)
        n.set_params(O.flatten(cfg, params))
        n.set_optimizer_state(np.zeros(n.n_params), np.zeros(n.n_params), 0, 0.9, 0.999)
        nets.append(n)
    for i, (B, upd, keep) in enumerate([(200, True, False), (200, True, False), (512, True, True),
                                        (200, False, True), (200, True, False), (512, True, False)]):
        x, lab = synthetic_batch(B, 2, seed=20 + i)
        res = [n.train_step(x, lab, update=upd, keep_grads=keep) for n in nets]
        assert res[0] == res[1], (i, res)
        if keep:
            np.testing.assert_array_equal(nets[0].get_grads(), nets[1].get_grads())
    np.testing.assert_array_equal(nets[0].get_params(), nets[1].get_params())
    s0, s1 = nets[0].get_optimizer_state(), nets[1].get_optimizer_state()
    for a, b in zip(s0, s1):
        np.testing.assert_array_equal(a, b)


def test_timers_cover_the_selected_kernel_classes_only():
    """lcn_set_timing with a set of classes: only those launches are timed,
    and the timers change nothing in the step's result."""
    from lcn_amd import native
    L, B = 2, 4096  # above the small-batch GEMM limit: the large kernels, colreduce path
    cfg, params, x, lab, net = _setup(dict(F=64, L=L, knn=3), B, seed=3)
    loss0, _ = net.train_step(x, lab, update=False)
    net.set_timing(True, only=[native.K_GEMM_DW, native.K_LIFT])
    loss1, _ = net.train_step(x, lab, update=False)
    n_dw, ms_dw, fl_dw = net.kernel_timing(native.K_GEMM_DW)
    assert n_dw == 2 * L and ms_dw > 0 and fl_dw == 2 * L * 2.0 * 4096.0 * 175 * B
    assert net.kernel_timing(native.K_LIFT)[0] == 1
    for k in (native.K_GEMM_FWD, native.K_GEMM_DX, native.K_BN_ACT, native.K_OUT, native.K_OUT_DW):
        assert net.kernel_timing(k)[0] == 0, k
    net.set_timing(True)
    net.train_step(x, lab, update=False)
    assert net.kernel_timing(native.K_GEMM_FWD)[0] == 2 * L
    assert net.kernel_timing(native.K_GEMM_DX)[0] == 2 * L
    net.set_timing(False)
    net.train_step(x, lab, update=False)
    assert net.kernel_timing(native.K_GEMM_DW)[0] == 0
    assert loss1 == loss0
    net.close()


def test_cfg4_full_batch_duplicated():
    """BASELINE.json configs[3] whole on one GPU: exponential mask, F 256, 6
    blocks, batch 131 072 as 65 536 poses taken twice.  Size-independent
    property (no oracle run at this size): the outputs of both halves equal
    those of the 65 536 batch, the loss and every gradient are unchanged
    (BN-parameter gradients with the looser bar of the 8 192 -> 16 384 case)."""
    cfg = make_cfg(F=256, L=6, knn=2, mask="exponential")
    params = perturbed_params(cfg)
    x, lab = synthetic_batch(65536, 2, seed=7)
    net = make_network(cfg, max_batch=131072)
    net.set_params(O.flatten(cfg, params))
    out1 = net.forward(x)
    l1, _ = net.train_step(x, lab, update=False, keep_grads=True)
    g1 = net.get_grads()
    x2, lab2 = np.concatenate([x, x]), np.concatenate([lab, lab])
    out2 = net.forward(x2)
    l2, _ = net.train_step(x2, lab2, update=False, keep_grads=True)
    g2 = net.get_grads()
    assert np.isfinite(out1).all() and np.isfinite(g1).all()
    np.testing.assert_array_equal(out2[:65536], out2[65536:])
    assert np.abs(out2[:65536] - out1).max() <= 1e-5
    assert l2 == pytest.approx(l1, rel=1e-6)
    for name, off, shape in net.param_layout():
        n = int(np.prod(shape))
        tol = 1e-3 if name.endswith(("_gamma", "_beta")) else 1e-4
        assert rel_err(g2[off:off + n], g1[off:off + n]) < tol, name
    net.close()
