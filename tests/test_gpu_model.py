"""The drop-in cgcnn (network/models_att.py surface) end to end on the MI355X:
fit / predict / evaluate / checkpoints / resume / TTA predict.

fit's arithmetic is the C-ABI train step (parity-tested against the oracle in
test_gpu_parity.py); here the bar is that fit drives it exactly as the
reference's loop does: the same permutation-deque batches (models_att.py:
193-200), evaluation every num_steps // num_epochs steps on the padded
validation batches, final/best checkpoints in the reference layout -- checked
bitwise against an explicit host-fed loop of lcn_train_step.
"""
import collections
import os
import shutil

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _params(dir_name, **over):
    from tools import filter_hub, params_help
    p = params_help.get_params(is_training=True)
    p.update(dict(dir_name=dir_name, num_epochs=2, batch_size=128, F=64, num_layers=2, knn=2,
                  init_type="same", dropout=0, mask_type="locally_connected"))
    p["neighbour_matrix"] = params_help.get_neighbour_matrix_by_hand(
        filter_hub.neighbour_dict_set[0], knn=2)
    p.update(over)
    return p


def _data(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1, 1, size=(n, 34))
    y = np.concatenate([x.reshape(n, 17, 2), rng.uniform(-1, 1, (n, 17, 1))], 2).reshape(n, 51)
    return x, y + 0.05 * rng.standard_normal(y.shape)


@pytest.fixture
def model_dir():
    name = "pytest_gpu_model"
    yield name
    from network import models_att
    shutil.rmtree(os.path.join(os.path.dirname(models_att.__file__), "..", "experiment", name),
                  ignore_errors=True)


def test_fit_predict_evaluate_checkpoints(model_dir, tmp_path):
    from network.models_att import cgcnn
    xtr, ytr = _data(640, 1)
    xva, yva = _data(300, 2)
    model = cgcnn(**_params(model_dir))
    net = model._net
    seen = []
    orig = net.train_step_indexed

    def spy(xs, ls, idx, **kw):
        if not seen:
            seen.append(net.get_params().copy())
        seen.append(np.array(idx).copy())
        return orig(xs, ls, idx, **kw)

    net.train_step_indexed = spy
    np.random.seed(5)
    losses, t_step = model.fit(xtr, ytr, xva, yva, output_dir=str(tmp_path))
    assert len(losses) == 2 and t_step > 0
    assert os.path.exists(tmp_path / "training_error.json")
    ck = model._get_path("checkpoints")
    for sub in ("final", "best"):
        assert os.path.exists(os.path.join(ck, sub, "checkpoint"))
    assert os.path.exists(os.path.join(ck, "final", "model-10.index"))
    assert os.path.exists(os.path.join(ck, "final", "model-10.data-00000-of-00001"))

    # the batches are the reference deque's
    np.random.seed(5)
    dq, ref_idx = collections.deque(), []
    for _ in range(10):
        if len(dq) < 128:
            dq.extend(np.random.permutation(640))
        ref_idx.append([dq.popleft() for _ in range(128)])
    for a, b in zip(seen[1:], ref_idx):
        np.testing.assert_array_equal(a, b)

    # the same steps fed from the host through lcn_train_step, bit for bit
    twin = cgcnn(**_params(model_dir + "_twin"))
    try:
        tn = twin._net
        tn.set_params(seen[0])
        tn.set_optimizer_state(np.zeros(tn.n_params), np.zeros(tn.n_params), 0, 0.9, 0.999)
        for idx in seen[1:]:
            tn.train_step(xtr[idx], ytr[idx])
        np.testing.assert_array_equal(tn.get_params(), net.get_params())
        # validation loss = predict with labels on the padded batches
        _, vloss = twin.predict(xva, yva, sess=tn)
        assert vloss == losses[-1]
    finally:
        shutil.rmtree(os.path.join(ck, "..", "..", model_dir + "_twin"), ignore_errors=True)

    # predict(sess=None) restores checkpoints/final, i.e. the end of fit
    p1 = model.predict(xva, sess=net)
    p0 = model.predict(xva)
    assert p0.dtype == np.float64 and p0.shape == (300, 51)
    np.testing.assert_array_equal(p0, p1)
    s, l = model.evaluate(xva, yva)
    assert s.startswith("loss:") and l == losses[-1]


def test_resume_keeps_restored_weights(model_dir):
    from network.models_att import cgcnn
    xtr, ytr = _data(256, 3)
    model = cgcnn(**_params(model_dir, num_epochs=1))
    np.random.seed(0)
    model.fit(xtr, ytr, xtr[:64], ytr[:64])
    ck = os.path.join(model._get_path("checkpoints"), "final")
    after = model._net.get_params().copy()
    m2 = cgcnn(**_params(model_dir, num_epochs=1))
    first = []
    orig = m2._net.train_step_indexed

    def spy(*a, **kw):
        if not first:
            first.append(m2._net.get_params().copy())
        return orig(*a, **kw)

    m2._net.train_step_indexed = spy
    # the reference resumes AT the checkpoint's step (range(starting_step, ...))
    m2.fit(xtr, ytr, xtr[:64], ytr[:64], starting_checkpoint=ck)
    assert len(first) == 1
    np.testing.assert_array_equal(first[0], after)


def test_predict_tta_matches_host_concatenation(model_dir):
    import lcn_oracle as O
    from network.models_att import cgcnn
    x, _ = _data(333, 4)
    model = cgcnn(**_params(model_dir, batch_size=100))
    net = model._net
    cat = np.concatenate([x, O.flip_data(x), O.rotate_data(x)], 0)
    ref = O.undo(model.predict(cat, sess=net), {"f": 1, "r": 2}, number_actions=2)
    got = model.predict_tta(x, flip=True, rotate=True, sess=net)
    assert np.abs(got - ref).max() <= 1e-5
    assert np.mean(np.abs(got - ref) <= 1e-12) > 0.99


def test_initialiser_on_the_librarys_own_layout():
    """init_flat fed from Network.param_layout() -- what cgcnn and bench.py do:
    the layout's names / offsets / shapes are the oracle's variable order, a
    bias comes out rank 1 (so cgcnn.kaiming's shape[0] is its own length,
    models_att.py:614-628: scale sqrt(2 / n), not sqrt(2)), and what is set is
    what the device holds."""
    import math
    import re

    import lcn_oracle as O
    from lcn_amd.init import init_flat
    from lcn_testutil import make_cfg, make_network
    cfg = make_cfg(F=64, L=2, knn=3)
    net = make_network(cfg, max_batch=32)
    layout = net.param_layout()
    off = 0
    for (name, o, shape), (oname, oshape) in zip(layout, O.param_specs(cfg)):
        assert (name, o, tuple(shape)) == (oname, off, tuple(oshape))
        off += int(np.prod(shape))
    assert off == net.n_params and len(layout) == len(O.param_specs(cfg))
    nb = O.neighbour_matrix(3)
    flat = init_flat(layout, net.n_params, nb, seed=5)
    n_bias = 0
    for name, o, shape in layout:
        v = flat[o:o + int(np.prod(shape))]
        if re.match(r"b\d", name):       # b1, b2_l, b3_l, b4 (not the bn* affine pairs)
            assert len(shape) == 1, (name, shape)
            s = math.sqrt(2.0 / shape[0])
            assert np.abs(v).max() <= 2.0 * s * (1 + 1e-6), name          # truncated at 2 sigma
            tol = 0.25 if v.size < 500 else 0.06
            assert abs(v.std() / (s * math.sqrt(0.77374)) - 1) < tol, (name, v.std(), s)
            n_bias += 1
        elif re.match(r"w\d", name):
            s = math.sqrt(2.0 / shape[0])
            assert len(shape) == 2 and np.abs(v).max() <= 2.0 * s * (1 + 1e-6), name
    assert n_bias == 2 * cfg.num_layers + 2
    net.set_params(flat)
    np.testing.assert_array_equal(net.get_params(), flat)
    net.close()
