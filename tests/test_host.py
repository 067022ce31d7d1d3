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


@pytest.mark.parametrize("tag,dt", [("f64", np.float64), ("f32", np.float32)])
def test_datareader_matches_reference_bitwise(golden_dir, tag, dt):
    """tools/data.py DataReader (read_2d / read_3d / denormalize) against the
    reference's own class on the same items (oracle/gen_golden.py)."""
    import gen_golden as G
    from tools import data
    g = np.load(os.path.join(golden_dir, "ref_datareader.npz"))
    tr, te = G.synthetic_gt(23, 1, dt), G.synthetic_gt(15, 2, dt)
    r = data.DataReader()
    x_tr, x_te = r.read_2d(tr, te)
    y_tr, y_te = r.read_3d()
    for name, got in (("x_train", x_tr), ("x_test", x_te), ("y_train", y_tr), ("y_test", y_te)):
        np.testing.assert_array_equal(got, g[f"{tag}_{name}"], err_msg=name)
    res = r.denormalize(g[f"{tag}_pred"])
    np.testing.assert_array_equal(np.stack([d["result"] for d in res]), g[f"{tag}_denorm"])
    keys = [f"{d['cameraid']}|{d['videoid']}|{d['subject']}|{d['action']}" for d in res]
    assert keys == list(g[f"{tag}_denorm_keys"])


def test_augmentation_helpers_match_reference(golden_dir):
    from tools import data
    g = np.load(os.path.join(golden_dir, "ref_helpers.npz"))
    np.testing.assert_array_equal(data.flip_data(g["flip_in2"]), g["flip_out2"])
    np.testing.assert_array_equal(data.flip_data(g["flip_in3"]), g["flip_out3"])
    np.testing.assert_array_equal(data.translation_data(g["trans_in2"], 0.07), g["trans_out2"])
    np.testing.assert_array_equal(data.translation_data(g["trans_in3"], -0.03), g["trans_out3"])
    np.testing.assert_allclose(data.rotate_data(g["rot_in2"], 180), g["rot_out2"], atol=1e-12)
    np.testing.assert_allclose(data.rotate_data(g["rot_in3"], 90), g["rot_out3_90"], atol=1e-12)
    np.testing.assert_allclose(data.undo(g["undo_in"], {"f": 1, "r": 2, "t": 3}, 3, translation=0.05),
                               g["undo_out_frt"], atol=1e-12)


# ---- one process per GPU: batch shards and shared seeds (lcn_amd/dist.py, cgcnn.fit) ----
def test_batch_shards_tile_the_batch():
    from lcn_amd import dist
    for total, world in ((200, 8), (512, 3), (65536, 8), (7, 7), (10, 4)):
        sl = [dist.shard_slice(total, world, r) for r in range(world)]
        assert sl[0].start == 0 and sl[-1].stop == total
        assert all(a.stop == b.start for a, b in zip(sl, sl[1:]))          # contiguous, in rank order
        sizes = [s.stop - s.start for s in sl]
        assert sizes == [dist.shard_rows(total, world, r) for r in range(world)]
        assert max(sizes) - min(sizes) <= 1
    # the ranks' slices of one drawn batch are exactly that batch, in order
    idx = np.random.permutation(1000)[:200]
    parts = [idx[dist.shard_slice(200, 3, r)] for r in range(3)]
    np.testing.assert_array_equal(np.concatenate(parts), idx)


class _SeedNet:
    """allreduce_host over fake ranks: sums what every rank contributes."""
    def __init__(self, contributions):
        self.contrib = contributions

    def allreduce_host(self, values, op="sum"):
        self.contrib.append(float(values[0]))
        return np.asarray([sum(self.contrib)])


def test_every_rank_draws_rank0s_seed_and_the_same_permutations():
    from network import models_att
    np.random.seed(123)
    expect = int(np.random.randint(0, 2 ** 31 - 1))
    np.random.seed(123)
    box = []
    s0 = models_att.shared_seed(_SeedNet(box), rank=0)        # rank 0 contributes its draw
    s1 = models_att.shared_seed(_SeedNet(box), rank=1)        # the others contribute 0
    assert s0 == s1 == expect
    draws = []
    for _ in range(2):                                         # two "ranks" reseed alike
        np.random.seed(s0)
        g = models_att.permutation_batches(50, 20)
        draws.append([next(g).copy() for _ in range(4)])
    for a, b in zip(*draws):
        np.testing.assert_array_equal(a, b)


def test_env_overrides_pick_device_and_transport(monkeypatch):
    from lcn_amd import dist
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert dist.dist_env() == (3, 4, 3)
    monkeypatch.setenv("LCN_DEVICE", "0")
    assert dist.dist_env() == (3, 4, 0)


def test_cli_flag_table_matches_the_reference_schema():
    """tools/cli_flags.py: flags, defaults, choices and required-ness of the
    two CLIs as the reference declares them (train.py:16-40, inference.py:16-40)."""
    from tools import cli_flags
    train = vars(cli_flags.parse("train", ["--train_set", "h36m", "--validation_set", "mpii"]))
    assert train == dict(
        test_indices="1", mask_type="locally_connected", init_type="same", knn=2, layers=3, dropout=0,
        channels=64, subset=None, epochs=25, batch_size=200, learning_rate=0.001, regularization=None,
        in_F=2, flip_data=False, rotation_data=False, translate_data=False, translation_factor=0.1,
        rotation_factor=60, resume_from=None, output_file=None, train_set="h36m",
        validation_set="mpii", test_set=None, n_test=1)
    inf = vars(cli_flags.parse("inference", ["--train_set", "h36m", "--test_set", "humansc3d"]))
    assert inf == dict(
        test_indices="1", mask_type="locally_connected", init_type="same", graph=0, knn=2, layers=3,
        in_joints=17, out_joints=17, dropout=0.25, channels=64, subset=None, epochs=200,
        checkpoints=None, batch_size=200, regularization=None, learning_rate=0.001, in_F=2,
        flip_data=False, rotation_data=False, translate_data=False, translation_factor=0.1,
        train_set="h36m", test_set="humansc3d")
    for prog, argv in (("train", ["--train_set", "h36m"]),                       # --validation_set required
                       ("inference", ["--train_set", "h36m"]),                   # --test_set required
                       ("train", ["--train_set", "h36m", "--validation_set", "h36m", "--init-type", "ones"]),
                       ("train", ["--train_set", "h36m", "--validation_set", "h36m", "--checkpoints", "best"]),
                       ("inference", ["--train_set", "x", "--test_set", "h36m"])):
        with pytest.raises(SystemExit):
            cli_flags.parse(prog, argv)
    ok = cli_flags.parse("inference", ["--train_set", "h36m", "--test_set", "h36m", "--init-type", "random",
                                       "--checkpoints", "best", "--flip-data", "--in-F", "3"])
    assert (ok.init_type, ok.checkpoints, ok.flip_data, ok.in_F) == ("random", "best", True, 3)
