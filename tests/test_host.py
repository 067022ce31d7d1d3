"""Host-side logic of the drop-in cgcnn that runs without a GPU."""
import collections
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lcn-pose_amd"))

from network.models_att import base_model, permutation_batches  # noqa: E402


def _reference_batches(n, bs, steps):
    """models_att.py:193-200 verbatim in behaviour: deque + popleft."""
    indices = collections.deque()
    out = []
    for _ in range(steps):
        if len(indices) < bs:
            indices.extend(np.random.permutation(n))
        out.append([indices.popleft() for _ in range(bs)])
    return out


@pytest.mark.parametrize("n,bs", [(1000, 256), (7, 3), (200, 200), (513, 64)])
def test_permutation_batches_follow_the_reference_deque(n, bs):
    steps = 3 * (n // bs + 2)
    np.random.seed(123)
    ref = _reference_batches(n, bs, steps)
    np.random.seed(123)
    gen = permutation_batches(n, bs)
    for r in ref:
        np.testing.assert_array_equal(next(gen), r)
    # the global numpy stream is left where the reference leaves it
    a = np.random.rand()
    np.random.seed(123)
    _reference_batches(n, bs, steps)
    assert np.random.rand() == a


def test_permutation_batches_bigger_than_the_dataset_fail_like_the_reference():
    with pytest.raises(IndexError):
        _reference_batches(5, 8, 1)
    with pytest.raises(IndexError):
        next(permutation_batches(5, 8))


def test_mean_batch_loss_is_float32_accumulation():
    m = base_model()
    m.batch_size = 200
    losses = np.array([0.1, 0.2, 0.30000001], np.float32)
    got = m._mean_batch_loss(losses, 550)
    ref = 0
    for l in losses:
        ref += l
    ref = ref * 200 / 550
    assert got == ref and np.asarray(got).dtype == np.asarray(ref).dtype
