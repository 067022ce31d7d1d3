"""The CPU oracle pinned against the reference's own outputs, then checked
for self-consistency (float64 finite differences, torch autograd)."""
import json
import os

import numpy as np
import pytest

import lcn_oracle as O


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


# --- pins against the reference's helpers and its own printed outputs --------

@pytest.mark.parametrize("knn", [1, 2, 3, 4, 5])
def test_neighbour_matrix_matches_reference_helper(golden_dir, knn):
    ref = _load(golden_dir, "ref_helpers.npz")[f"neighbour_knn{knn}"]
    np.testing.assert_array_equal(O.neighbour_matrix(knn), ref)


def test_neighbour_matrix_matches_notebook_dumps(golden_dir):
    nb = _load(golden_dir, "notebook_masks.npz")
    np.testing.assert_array_equal(O.neighbour_matrix(2), nb["nb_h36m_knn2"])
    np.testing.assert_array_equal(O.neighbour_matrix(1), nb["nb_humansc3d_knn1"])


def test_block_counts():
    # nnz 57/111/175/273 for knn 1/2/3/5
    for knn, nnz in ((1, 57), (2, 111), (3, 175), (5, 273)):
        assert int(O.neighbour_matrix(knn).sum()) == nnz


def test_exponential_matrix_matches_reference_helper(golden_dir):
    ref = _load(golden_dir, "ref_helpers.npz")["exp_matrix"]
    np.testing.assert_array_equal(O.exponential_matrix(), ref)


def test_tta_helpers_match_reference(golden_dir):
    g = _load(golden_dir, "ref_helpers.npz")
    np.testing.assert_allclose(O.flip_data(g["flip_in2"]), g["flip_out2"], rtol=0, atol=0)
    np.testing.assert_allclose(O.flip_data(g["flip_in3"]), g["flip_out3"], rtol=0, atol=0)
    np.testing.assert_allclose(O.rotate_data(g["rot_in2"], 180), g["rot_out2"], atol=1e-12)
    np.testing.assert_allclose(O.rotate_data(g["rot_in3"], 180), g["rot_out3"], atol=1e-12)
    np.testing.assert_allclose(O.rotate_data(g["rot_in3"], 90), g["rot_out3_90"], atol=1e-12)
    np.testing.assert_allclose(O.undo(g["undo_in"][:15], {"f": 1, "r": 2}, 2), g["undo_out_fr"],
                               atol=1e-12)
    np.testing.assert_allclose(O.undo(g["undo_in"], {"f": 1, "r": 2, "t": 3}, 3, translation=0.05),
                               g["undo_out_frt"], atol=1e-12)
    np.testing.assert_array_equal(O.translation_data(g["trans_in2"], 0.07), g["trans_out2"])
    np.testing.assert_array_equal(O.translation_data(g["trans_in3"], -0.03), g["trans_out3"])
    np.testing.assert_allclose(O.rotate_data(g["trans_in2"], 37.0), g["rot_out2_37"], atol=1e-12)


def test_learning_rate_matches_notebook_logs(golden_dir):
    facts = json.load(open(os.path.join(golden_dir, "notebook_facts.json")))
    cfg = O.Config()
    # the logged value is formatted "{:.2e}"; the op reads global_step before the increment
    assert float(f"{O.learning_rate(cfg, facts['h36m_step1'] - 1):.2e}") == facts["h36m_lr1"]
    assert float(f"{O.learning_rate(cfg, facts['sc3d_step1'] - 1):.2e}") == facts["sc3d_lr1"]
    # models_att.py:185-186: num_steps = int(epochs*N/B), eval_frequency = num_steps // epochs
    N = facts["h36m_total_steps"]  # B=200, epochs=200 -> num_steps == N
    assert int(facts["h36m_epochs"] * N / facts["h36m_batch"]) == facts["h36m_total_steps"]
    assert facts["h36m_total_steps"] // facts["h36m_epochs"] == facts["h36m_step1"]
    assert facts["sc3d_total_steps"] // facts["sc3d_epochs"] == facts["sc3d_step1"]


# --- oracle regression pins ---------------------------------------------------

@pytest.mark.parametrize("name", ["lc_knn3_F8_L2_B24", "lc_knn1_F8_L1_B16_in3", "exp_F8_L1_B16",
                                  "lc_knn3_F64_L3_B32"])
def test_oracle_reproduces_fixture(golden_dir, name):
    d = _load(golden_dir, f"oracle_{name}.npz")
    c = json.loads(str(d["meta"]))
    cfg = O.Config(F=c["F"], in_F=c["in_F"], num_layers=c["L"], mask_type=c["mask"],
                   neighbour=O.neighbour_matrix(c["knn"]))
    params = O.init_params(cfg, seed=1)
    out, cache = O.forward(cfg, params, d["x"], np.float64)
    np.testing.assert_allclose(out, d["out"], rtol=1e-12, atol=1e-12)
    grads = O.backward(cfg, params, cache, d["lab"], np.float64)
    flat = np.concatenate([grads[n].ravel() for n, _ in O.param_specs(cfg)])
    if "grads_flat" in d:
        np.testing.assert_allclose(O.flatten(cfg, params), d["params_flat"], rtol=0, atol=0)
        np.testing.assert_allclose(flat, d["grads_flat"], rtol=1e-10, atol=1e-14)
    else:
        sel = d["sample_idx"]
        np.testing.assert_allclose(O.flatten(cfg, params)[sel], d["params_flat_sample"], rtol=0)
        np.testing.assert_allclose(flat[sel], d["grads_flat_sample"], rtol=1e-10, atol=1e-14)


# --- self-consistency ----------------------------------------------------------

def _small_cfg(mask="locally_connected", **kw):
    return O.Config(F=kw.pop("F", 4), in_F=kw.pop("in_F", 2), num_layers=kw.pop("L", 1),
                    mask_type=mask, neighbour=O.neighbour_matrix(kw.pop("knn", 2)), **kw)


@pytest.mark.parametrize("mask,kw", [("locally_connected", {}),
                                     ("exponential", {}),
                                     ("locally_connected", {"residual": False, "in_F": 3}),
                                     ("locally_connected", {"batch_norm": False}),
                                     ("locally_connected", {"regularization": 0.01}),
                                     ("locally_connected", {"dropout": (0.3, 77, 2)})])
def test_backward_matches_finite_differences(mask, kw):
    drop = kw.pop("dropout", None)
    cfg = _small_cfg(mask, **kw)
    params = {k: v.astype(np.float64) for k, v in O.init_params(cfg, seed=5).items()}
    if "mask" in params:  # break the symmetric init so softmax gradients are generic
        params["mask"] = params["mask"] + np.random.default_rng(9).normal(0, 0.3, (17, 17))
    rng = np.random.default_rng(4)
    B = 6
    x = rng.uniform(-1, 1, size=(B, 17 * cfg.in_F))
    lab = rng.uniform(-1, 1, size=(B, 51))

    def loss_of(p):
        out, _ = O.forward(cfg, p, x, np.float64, drop=drop)
        return O.mse_loss(out, lab) + O.reg_loss(cfg, p)

    out, cache = O.forward(cfg, params, x, np.float64, drop=drop)
    grads = O.backward(cfg, params, cache, lab, np.float64)
    rs = np.random.default_rng(11)
    for name, shape in O.param_specs(cfg):
        g = grads[name]
        for _ in range(4):
            idx = tuple(rs.integers(0, s) for s in shape)
            h = 1e-6
            p1 = {k: v.copy() for k, v in params.items()}
            p2 = {k: v.copy() for k, v in params.items()}
            p1[name][idx] += h
            p2[name][idx] -= h
            fd = (loss_of(p1) - loss_of(p2)) / (2 * h)
            assert abs(fd - g[idx]) <= 1e-6 + 1e-4 * abs(fd), (name, idx, fd, g[idx])


def test_backward_matches_torch_autograd():
    torch = pytest.importorskip("torch")
    cfg = _small_cfg("locally_connected", F=8, L=2, knn=3)
    params = O.init_params(cfg, seed=3)
    params["mask"] = params["mask"] + np.random.default_rng(1).normal(0, 0.5, (17, 17)).astype(np.float32)
    rng = np.random.default_rng(0)
    B = 12
    x = rng.uniform(-1, 1, size=(B, 34))
    lab = rng.uniform(-1, 1, size=(B, 51))
    out, cache = O.forward(cfg, params, x, np.float64)
    grads = O.backward(cfg, params, cache, lab, np.float64)

    T = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in params.items()}
    C = torch.tensor(O.structure(cfg), dtype=torch.float64)
    M = torch.softmax(T["mask"], dim=0) * C
    xt = torch.tensor(x)

    def lin(a, wn, bn, fin, fout):
        W = T[wn]
        n = torch.linalg.norm(W)
        Wc = W / torch.clamp(n, min=1.0)
        We = (Wc.reshape(17, fin, 17, fout) * M.reshape(17, 1, 17, 1)).reshape(W.shape)
        return a @ We + T[bn]

    def bnact(z, pre, F):
        z3 = z.reshape(z.shape[0], 17, F)
        mu = z3.mean(dim=(0, 1))
        var = ((z3 - mu) ** 2).mean(dim=(0, 1))
        inv = T[pre + "_gamma"] / torch.sqrt(var + 1e-3)
        u = (z3 * inv + (T[pre + "_beta"] - mu * inv)).reshape(z.shape)
        return torch.where(u > 0, u, 0.2 * u)

    h = bnact(lin(xt, "w1", "b1", 2, 8), "bn0", 8)
    for l in range(cfg.num_layers):
        g = bnact(lin(h, f"w2_{l}", f"b2_{l}", 8, 8), f"bn1{l}", 8)
        t = bnact(lin(g, f"w3_{l}", f"b3_{l}", 8, 8), f"bn2{l}", 8)
        h = h + t
    y = lin(h, "w4", "b4", 8, 3).reshape(B, 17, 3)
    x3 = xt.reshape(B, 17, 2)
    o = torch.cat([x3 + y[:, :, :2], y[:, :, 2:3]], dim=2).reshape(B, 51)
    loss = ((o - torch.tensor(lab)) ** 2).mean()
    loss.backward()
    np.testing.assert_allclose(o.detach().numpy(), out, rtol=1e-12, atol=1e-12)
    for name, _ in O.param_specs(cfg):
        np.testing.assert_allclose(grads[name], T[name].grad.numpy(), rtol=1e-9, atol=1e-13,
                                   err_msg=name)


def test_fp32_forward_close_to_fp64():
    cfg = O.Config(F=64, num_layers=3, neighbour=O.neighbour_matrix(3))
    params = O.init_params(cfg, seed=0)
    x = np.random.default_rng(0).uniform(-1, 1, (64, 34)).astype(np.float32)
    o32, _ = O.forward(cfg, params, x, np.float32)
    o64, _ = O.forward(cfg, params, x, np.float64)
    assert np.abs(o32 - o64).max() < 1e-4


def test_adam_matches_closed_form():
    cfg = _small_cfg()
    params = {"a": np.array([1.0, -2.0], np.float32)}
    st = O.AdamState({"a": np.zeros(2, np.float32)}, {"a": np.zeros(2, np.float32)})
    g = {"a": np.array([0.5, -0.25], np.float32)}
    lr = O.adam_step(cfg, params, g, st)
    assert lr == np.float32(1e-3)
    # first step: m = 0.1 g, v = 0.001 g^2, alpha = lr*sqrt(0.001)/0.1 -> step = lr*sign(g)
    np.testing.assert_allclose(params["a"], [1.0 - 1e-3, -2.0 + 1e-3], rtol=1e-5)
    assert st.global_step == 1 and st.beta1_power == np.float32(0.9) * np.float32(0.9)


def test_dropout_masks():
    """Counter-based dropout masks (lcn_internal.h Dropout): the kept fraction
    is 1 - rate, masks differ across layers, steps, seeds and rows, and
    rate 0 keeps everything; the scale is TF's float32 1 / (1 - rate)."""
    B, H = 512, 1088
    for rate in (0.25, 0.3, 0.5):
        m = O.dropout_mask(rate, 123, 0, 1, B, H)
        assert abs(m.mean() - (1 - rate)) < 4 * np.sqrt(rate * (1 - rate) / m.size)
    a = O.dropout_mask(0.3, 123, 0, 1, B, H)
    for other in (O.dropout_mask(0.3, 123, 0, 2, B, H), O.dropout_mask(0.3, 123, 1, 1, B, H),
                  O.dropout_mask(0.3, 124, 0, 1, B, H), O.dropout_mask(0.3, 123, 0, 1, B, H, row0=B)):
        agree = (a == other).mean()
        assert abs(agree - (0.7 ** 2 + 0.3 ** 2)) < 0.01, agree   # independent masks
    assert O.dropout_mask(0.0, 5, 3, 0, 8, 64).all()
    assert O.dropout_scale(0.3) == np.float32(1) / (np.float32(1) - np.float32(0.3))
    # row0 shifts rows: the second half of a 2B batch is the B batch at row0 = B
    np.testing.assert_array_equal(O.dropout_mask(0.3, 9, 4, 3, 2 * B, H)[B:],
                                  O.dropout_mask(0.3, 9, 4, 3, B, H, row0=B))
