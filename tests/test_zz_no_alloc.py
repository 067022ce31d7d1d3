"""lcn_eval_mpjpe_static, the allocation-free variant of lcn_eval_mpjpe (its
device staging lives in a fixed per-GPU array of the library): through the C
ABI, against lcn_eval_mpjpe on the same frames -- bit for bit, both kernels
being the same code -- on two calls in a row, the second with fewer frames
(the array keeps the first call's contents), then its size limit."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_f64p = ctypes.POINTER(ctypes.c_double)


def _frames(n, seed):
    rng = np.random.default_rng(seed)
    gt = rng.normal(0, 400, (n, 17, 3)) + np.array([0, 0, 4500.0])
    pred = np.empty((n, 17, 3))
    pred[:, :, :2] = rng.uniform(100, 900, (n, 17, 2))
    pred[:, :, 2] = rng.normal(0, 300, (n, 17))
    box = np.concatenate([rng.uniform(0, 300, (n, 2)), rng.uniform(600, 1000, (n, 2))], axis=1)
    cam = np.concatenate([rng.uniform(480, 540, (n, 2)), rng.uniform(1100, 1200, (n, 2))], axis=1)
    root = rng.uniform(3000, 6000, n)
    return pred, gt, box, cam, root


def _call(lib, fn, arrs, proto, n=None):
    arrs = [np.ascontiguousarray(a, np.float64) for a in arrs]
    n = arrs[0].shape[0] if n is None else n
    err = np.full((max(n, 1), 17), np.nan)
    rc = fn(0, n, *[a.ctypes.data_as(_f64p) for a in arrs], proto, err.ctypes.data_as(_f64p))
    return rc, err[:n]


@pytest.mark.parametrize("proto", [0, 1], ids=["protocol1", "protocol2"])
def test_static_entry_point_equals_the_allocating_one_on_two_calls_in_a_row(proto):
    from lcn_amd import native
    lib = native.load_library()
    for n, seed in ((5000, 1), (1200, 2)):     # the second call is smaller: stale rows stay behind it
        arrs = _frames(n, seed)
        rc_a, want = _call(lib, lib.lcn_eval_mpjpe, arrs, proto)
        rc_s, got = _call(lib, lib.lcn_eval_mpjpe_static, arrs, proto)
        assert rc_a == 0 and rc_s == 0, lib.lcn_last_error(None)
        assert np.isfinite(want).all()
        np.testing.assert_array_equal(got, want)
    # the Python wrapper takes the same route
    arrs = _frames(300, 3)
    np.testing.assert_array_equal(native.eval_mpjpe(*arrs, protocol2=bool(proto), static=True),
                                  native.eval_mpjpe(*arrs, protocol2=bool(proto)))


def test_static_entry_point_limits_and_edges():
    from lcn_amd import native
    lib = native.load_library()
    cap = native.EVAL_STATIC_MAX_FRAMES
    arrs = _frames(cap, 4)
    rc, got = _call(lib, lib.lcn_eval_mpjpe_static, arrs, 0)          # exactly the limit
    assert rc == 0
    np.testing.assert_array_equal(got, _call(lib, lib.lcn_eval_mpjpe, arrs, 0)[1])
    big = _frames(cap + 1, 5)
    rc, _ = _call(lib, lib.lcn_eval_mpjpe_static, big, 0)             # one frame more: refused
    assert rc == -1 and b"exceed the static limit" in lib.lcn_last_error(None)
    rc, _ = _call(lib, lib.lcn_eval_mpjpe_static, arrs, 0, n=0)       # nothing to do
    assert rc == 0
    rc = lib.lcn_eval_mpjpe_static(0, 5, None, None, None, None, None, 0, None)
    assert rc == -1 and b"null" in lib.lcn_last_error(None)
    with pytest.raises(native.LcnNativeError, match="static limit"):
        native.eval_mpjpe(*big, static=True)
