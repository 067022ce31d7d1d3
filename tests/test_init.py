"""lcn_amd.init: the product's only initialiser for fit (cgcnn._initialize),
against cgcnn.kaiming and the variable initial values of the reference graph
(models_att.py:614-628 kaiming; :557-566 mask = L; Keras BatchNormalization
gamma = 1, beta = 0).  TF's stream cannot be reproduced (unseeded), so the
distribution is what is checked."""
import math

import numpy as np

import lcn_oracle as O
from lcn_amd.init import init_flat, truncated_normal
from lcn_testutil import make_cfg


def _layout(cfg):
    out, off = [], 0
    for name, shape in O.param_specs(cfg):
        out.append((name, off, tuple(shape)))
        off += int(np.prod(shape))
    return out, off


def test_truncated_normal_is_resampled_within_two_sigma():
    rng = np.random.default_rng(0)
    v = truncated_normal(rng, (400, 500))
    assert np.abs(v).max() <= 2.0
    # tf.random.truncated_normal(stddev=1): a standard normal conditioned on
    # |x| <= 2 has variance 1 - 4 phi(2) / (2 Phi(2) - 1) = 0.7737
    assert abs(v.mean()) < 5e-3 and abs(v.var() - 0.77374) < 5e-3
    # resampled, not clipped: no mass piled at the bounds
    assert (np.abs(v) > 1.999).mean() < 1e-3


def test_kaiming_scale_per_tensor_including_biases():
    cfg = make_cfg(F=64, L=2, knn=3)
    layout, n = _layout(cfg)
    nb = O.neighbour_matrix(3)
    flat = init_flat(layout, n, nb, seed=1)
    assert flat.dtype == np.float32 and flat.shape == (n,) and np.isfinite(flat).all()
    seen = set()
    for name, off, shape in layout:
        v = flat[off:off + int(np.prod(shape))].reshape(shape)
        if name == "mask":
            np.testing.assert_array_equal(v, nb.T.astype(np.float32))       # V = L = N^T (:549, :557)
        elif name.endswith("_gamma"):
            np.testing.assert_array_equal(v, 1.0)
        elif name.endswith("_beta"):
            np.testing.assert_array_equal(v, 0.0)
        else:
            # truncated_normal * sqrt(2 / shape[0]); a bias is rank 1, so its
            # shape[0] is its own length (:614-628)
            s = math.sqrt(2.0 / shape[0])
            assert np.abs(v).max() <= 2.0 * s * (1 + 1e-6), name
            want = s * math.sqrt(0.77374)
            tol = 0.2 if v.size < 500 else 0.05
            assert abs(v.std() / want - 1) < tol, (name, v.std(), want)
            seen.add(name[0])
    assert seen == {"w", "b"}
    # weights are dense: entries outside the mask's support are initialised too
    w2 = dict((nm, (o, sh)) for nm, o, sh in layout)["w2_0"]
    blk = flat[w2[0]:w2[0] + int(np.prod(w2[1]))].reshape(17, 64, 17, 64)
    assert np.abs(blk[3, :, 16, :]).min() >= 0 and np.abs(blk[3, :, 16, :]).max() > 0   # joints 3, 16 unconnected


def test_seed_and_layout_follow_the_library_order():
    cfg = make_cfg(F=64, L=1, knn=2)
    layout, n = _layout(cfg)
    nb = O.neighbour_matrix(2)
    a, b = init_flat(layout, n, nb, seed=7), init_flat(layout, n, nb, seed=7)
    np.testing.assert_array_equal(a, b)
    assert not np.array_equal(a, init_flat(layout, n, nb, seed=8))
    # the exponential mask has no trainable mask variable
    cfg_e = make_cfg(F=64, L=1, mask="exponential")
    assert "mask" not in [nm for nm, _ in O.param_specs(cfg_e)]
    le, ne = _layout(cfg_e)
    assert init_flat(le, ne, nb, seed=0).shape == (ne,)
