"""Device-resident datasets on the MI355X: permutation
gather, fixed-batch predict with zero padding, test-time augmentation.

Bars: the gathered batch is bit-identical to the reference's host path
(fancy-index the float64 arrays, cast to float32 at the feed); a step or a
predict on the gathered batch is bit-identical to the same step on the
host-fed batch (same kernels, same input bits); augmented copies are
bit-identical to the oracle's float64 restatement of tools/data.py cast to
float32 (rotation: at most 1 ulp on a vanishing fraction, FMA order of the
2x2 product); the undone + averaged predictions agree with oracle.undo to
1e-12 (float64 arithmetic, same order).
"""
import numpy as np
import pytest

import lcn_oracle as O
from lcn_testutil import make_cfg, make_network, perturbed_params

pytestmark = pytest.mark.gpu

X_SLOT, L_SLOT = 0, 1


def _data(N, in_F=2, seed=5):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1, 1, size=(N, 17 * in_F))          # float64, as DataReader yields
    lab = rng.uniform(-1, 1, size=(N, 51))
    return x, lab


def _net(B, in_F=2, **kw):
    cfg = make_cfg(F=64, L=2, knn=3, in_F=in_F, **kw)
    params = perturbed_params(cfg, seed=3)
    net = make_network(cfg, max_batch=B)
    net.set_params(O.flatten(cfg, params))
    net.set_optimizer_state(np.zeros(net.n_params), np.zeros(net.n_params), 0, 0.9, 0.999)
    return cfg, params, net


def test_gathered_batch_is_the_host_feed():
    N, B = 1000, 300
    x, lab = _data(N)
    _, _, net = _net(B)
    net.dataset_upload(X_SLOT, x)
    net.dataset_upload(L_SLOT, lab)
    idx = np.random.default_rng(0).permutation(N)[:B]
    net.train_step_indexed(X_SLOT, L_SLOT, idx, update=False)
    got_x = net.debug_tensor(5, 0, B * 34).reshape(B, 34)
    got_l = net.debug_tensor(6, 0, B * 51).reshape(B, 51)
    np.testing.assert_array_equal(got_x, x[idx].astype(np.float32))
    np.testing.assert_array_equal(got_l, lab[idx].astype(np.float32))


def test_indexed_steps_equal_host_steps():
    N, B = 900, 256
    x, lab = _data(N, seed=6)
    _, _, a = _net(B)
    _, _, b = _net(B)
    b.dataset_upload(X_SLOT, x)
    b.dataset_upload(L_SLOT, lab)
    rng = np.random.default_rng(1)
    for _ in range(3):
        idx = rng.permutation(N)[:B]
        la, lra = a.train_step(x[idx], lab[idx])
        lb, lrb = b.train_step_indexed(X_SLOT, L_SLOT, idx)
        assert la == lb and lra == lrb
    np.testing.assert_array_equal(a.get_params(), b.get_params())
    ma, va, *_ = a.get_optimizer_state()
    mb, vb, *_ = b.get_optimizer_state()
    np.testing.assert_array_equal(ma, mb)
    np.testing.assert_array_equal(va, vb)


def test_device_index_pointer():
    N, B = 512, 128
    x, lab = _data(N, seed=7)
    _, _, a = _net(B)
    _, _, b = _net(B)
    for n in (a, b):
        n.dataset_upload(X_SLOT, x)
        n.dataset_upload(L_SLOT, lab)
    idx = np.random.default_rng(2).permutation(N).astype(np.int32)
    buf = b.device_buffer(0, idx.nbytes)
    buf.upload(idx)
    la, _ = a.train_step_indexed(X_SLOT, L_SLOT, idx[128:256])
    lb, _ = b.train_step_indexed(X_SLOT, L_SLOT, None, idx_device_ptr=buf.ptr + 128 * 4, batch=B)
    assert la == lb
    np.testing.assert_array_equal(a.get_params(), b.get_params())


def _host_predict(net, data, bs, labels=None):
    """models_att.py:79-132 with host feeds (fixed batches, zero padding)."""
    size = data.shape[0]
    preds = np.empty((size, 51))
    losses = []
    for begin in range(0, size, bs):
        end = min(begin + bs, size)
        bd = np.zeros((bs, data.shape[1]), np.float32)
        bd[: end - begin] = data[begin:end]
        if labels is not None:
            bl = np.zeros((bs, 51), np.float32)
            bl[: end - begin] = labels[begin:end]
            p, l = net.forward_loss(bd, bl)
            losses.append(l)
        else:
            p = net.forward(bd)
        preds[begin:end] = p[: end - begin]
    return preds, np.array(losses, np.float32)


@pytest.mark.parametrize("N,bs", [(1000, 256), (256, 256), (37, 64)])
def test_predict_dataset_equals_host_predict(N, bs):
    x, lab = _data(N, seed=8)
    _, _, net = _net(bs)
    net.dataset_upload(X_SLOT, x)
    net.dataset_upload(L_SLOT, lab)
    ref, ref_losses = _host_predict(net, x, bs, lab)
    got, losses = net.predict_dataset(X_SLOT, N, bs, lab_slot=L_SLOT)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(losses, ref_losses)
    got2 = net.predict_dataset(X_SLOT, N, bs)
    np.testing.assert_array_equal(got2, ref)


def _ulps(a, b):
    ai = a.astype(np.float32).view(np.int32).astype(np.int64)
    bi = b.astype(np.float32).view(np.int32).astype(np.int64)
    return np.abs(ai - bi)


@pytest.mark.parametrize("in_F", [2, 3])
@pytest.mark.parametrize("op", ["flip", "rot180", "rot37", "trans"])
def test_augmented_copy_matches_reference_helpers(op, in_F):
    from lcn_amd.native import AUG_FLIP, AUG_NONE, AUG_ROTATE, AUG_TRANSLATE
    N = 120
    x, _ = _data(N, in_F=in_F, seed=9)
    _, _, net = _net(256, in_F=in_F)
    net.dataset_upload(X_SLOT, x)
    if op == "flip":
        ref, a = O.flip_data(x), (AUG_FLIP, 0.0, 0.0)
    elif op.startswith("rot"):
        ang = float(op[3:])
        th = np.radians(ang)
        ref, a = O.rotate_data(x, ang), (AUG_ROTATE, float(np.cos(th)), float(np.sin(th)))
    else:
        ref, a = O.translation_data(x, 0.07), (AUG_TRANSLATE, 0.07, 0.0)
    ops = [(AUG_NONE, 0.0, 0.0), a]
    net.predict_dataset(X_SLOT, N, 256, augment=ops, undo=ops)  # one batch: [x; op(x); zeros]
    got = net.debug_tensor(5, 0, 256 * 17 * in_F).reshape(256, 17 * in_F)
    np.testing.assert_array_equal(got[:N], x.astype(np.float32))
    np.testing.assert_array_equal(got[2 * N:], 0)
    d = _ulps(got[N:2 * N], ref.astype(np.float32))
    if op.startswith("rot"):
        assert d.max() <= 1 and (d > 0).mean() < 1e-2, (d.max(), (d > 0).mean())
    else:
        assert d.max() == 0


@pytest.mark.parametrize("flags", [("f",), ("f", "r"), ("f", "r", "t"), ("r", "t")])
def test_tta_predict_matches_inference_pipeline(flags):
    """inference.py:70-110: concat copies -> predict -> data.undo, against the
    device path that never concatenates."""
    from lcn_amd.tta import augment_ops
    N, bs = 700, 256
    x, _ = _data(N, seed=10)
    _, _, net = _net(bs)
    t = 0.043 if "t" in flags else None
    aug, undo, op_ord = augment_ops(flip="f" in flags, rotate="r" in flags, translation=t)
    cat = [x]
    if "f" in flags:
        cat.append(O.flip_data(x))
    if "r" in flags:
        cat.append(O.rotate_data(x))
    if "t" in flags:
        cat.append(O.translation_data(x, t))
    preds, _ = _host_predict(net, np.concatenate(cat, axis=0), bs)
    ref = O.undo(preds, op_ord, number_actions=len(cat) - 1, translation=t if t else 0.5)
    net.dataset_upload(X_SLOT, x)
    got = net.predict_dataset(X_SLOT, N, bs, augment=aug, undo=undo)
    # the only possible difference: a rotated input 1 ulp apart (FMA order of
    # the 2x2 product) moves that pose's prediction by float32 rounding noise
    assert np.abs(got - ref).max() <= 1e-5
    assert np.mean(np.abs(got - ref) <= 1e-12) > 0.99


def test_cfg5_share_tta_predict_full_size():
    """BASELINE.json configs[4] at one GPU's share of its 8-GPU batch: knn 5,
    3 blocks, 32 768 poses x 3 TTA copies (flip + rotation) = 98 304 network
    rows in batches of 32 768.  Size-independent checks, no oracle run:
    (a) the device TTA path equals the inference.py pipeline fed from the host
    (concatenate the copies, fixed-batch predict, data.undo, inference.py:70-111);
    (b) a dataset holding every pose twice, predicted in batches twice as
    large, gives each pose the same prediction as before -- in both halves
    (batch-statistics BN and the undo / mean are invariant to duplication)."""
    from lcn_amd.tta import augment_ops
    N, bs = 32768, 32768
    cfg = make_cfg(F=64, L=3, knn=5)
    net = make_network(cfg, max_batch=2 * bs)
    net.set_params(O.flatten(cfg, perturbed_params(cfg, seed=9)))
    x, _ = _data(N, seed=12)
    aug, undo, op_ord = augment_ops(flip=True, rotate=True)
    net.dataset_upload(X_SLOT, x)
    got = net.predict_dataset(X_SLOT, N, bs, augment=aug, undo=undo)
    assert got.shape == (N, 51) and np.isfinite(got).all()
    # (a) host-fed copies through the same network
    cat = np.concatenate([x, O.flip_data(x), O.rotate_data(x)], axis=0)
    preds, _ = _host_predict(net, cat, bs)
    ref = O.undo(preds, op_ord, number_actions=2, translation=0.5)
    assert np.abs(got - ref).max() <= 1e-5
    assert np.mean(np.abs(got - ref) <= 1e-12) > 0.99
    # (b) every pose twice, batches twice as large
    net.dataset_upload(X_SLOT, np.concatenate([x, x], axis=0))
    dup = net.predict_dataset(X_SLOT, 2 * N, 2 * bs, augment=aug, undo=undo)
    np.testing.assert_array_equal(dup[:N], dup[N:])
    assert np.abs(dup[:N] - got).max() <= 1e-5
    net.close()
