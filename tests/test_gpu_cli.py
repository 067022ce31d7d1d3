"""train.py / inference.py (the reference's CLIs, train.py:12-121 and
inference.py:12-127) end to end on the MI355X, on synthetic pickled datasets
this test writes (the reference's per-frame dict schema)."""
import os
import pickle
import shutil
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "lcn-pose_amd")


@pytest.fixture
def dataset(tmp_path):
    import gen_golden as G
    for split, n, seed in (("train", 512, 1), ("val", 150, 2), ("test", 130, 3)):
        with open(tmp_path / f"h36m_{split}.pkl", "wb") as f:
            pickle.dump(G.synthetic_gt(n, seed, np.float64), f)
    yield str(tmp_path)
    shutil.rmtree(os.path.join(PKG, "experiment", "test97"), ignore_errors=True)


def _run(args, env_dir):
    env = dict(os.environ, LCN_DATASET_DIR=env_dir, PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable] + args, cwd=PKG, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_train_then_inference_with_tta(dataset):
    common = ["--test-indices", "97", "--knn", "2", "--layers", "1", "--batch_size", "64"]
    out = _run(["train.py", "--train_set", "h36m", "--validation_set", "h36m", "--epochs", "2"]
               + common, dataset)
    assert "Total steps to be done to complete all the epochs: 16" in out
    ck = os.path.join(PKG, "experiment", "test97", "checkpoints")
    assert os.path.exists(os.path.join(ck, "best", "checkpoint"))
    assert os.path.exists(os.path.join(ck, "final", "model-16.index"))

    _run(["inference.py", "--train_set", "h36m", "--test_set", "h36m", "--checkpoints", "final",
          "--flip-data", "--rotation-data"] + common, dataset)
    res = pickle.load(open(os.path.join(PKG, "experiment", "test97", "result.pkl"), "rb"))
    assert len(res) == 130 and res[0]["result"].shape == (17, 3)

    # the same pipeline through the Python API with host-side TTA (inference.py's
    # own concatenate -> predict -> undo), restored from the same checkpoint
    sys.path.insert(0, PKG)
    from network.models_att import cgcnn
    from tools import data, params_help
    import argparse
    args = argparse.Namespace(test_indices="97", knn=2, layers=1, dropout=0.25, channels=64,
                              checkpoints="final", mask_type="locally_connected",
                              init_type="same", epochs=200, batch_size=64,
                              learning_rate=0.001, regularization=None)
    params = params_help.get_params(is_training=True, gt_dataset=None)
    params_help.update_parameters(args, params)
    r = data.DataReader()
    os.environ["LCN_DATASET_DIR"] = dataset
    _, test = r.read_2d(r.real_read("h36m", "train"), r.real_read("h36m", "test"))
    model = cgcnn(**params)
    cat = np.concatenate([test, data.flip_data(test.copy()), data.rotate_data(test.copy())], 0)
    preds = data.undo(model.predict(cat), {"f": 1, "r": 2}, number_actions=2)
    ref = np.stack([d["result"] for d in r.denormalize(preds)])
    got = np.stack([d["result"] for d in res])
    # pixels: float32 network noise of a 1-ulp rotated input at most
    assert np.abs(got - ref).max() < 1e-2
    assert np.mean(np.abs(got - ref) < 1e-9) > 0.99
