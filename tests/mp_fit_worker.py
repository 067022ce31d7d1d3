"""One rank of a cgcnn.fit run for tests/test_gpu_multiproc.py (not a test).

usage: mp_fit_worker.py OUT.npz   (RANK / WORLD_SIZE / LCN_* from the environment)
Trains a small LCN on synthetic poses for two epochs and saves the
validation losses, t_step-independent results and the final parameters."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "lcn-pose_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

from lcn_testutil import synthetic_batch  # noqa: E402
from network import models_att  # noqa: E402
from tools import params_help  # noqa: E402
from tools.filter_hub import neighbour_dict_set  # noqa: E402


def main(out):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    x, lab = synthetic_batch(700, seed=3)
    tx, tl, vx, vl = x[:600].astype(np.float64), lab[:600].astype(np.float64), \
        x[600:].astype(np.float64), lab[600:].astype(np.float64)
    np.random.seed(5)
    if world == 1:
        # what a multi-rank fit does to the permutation stream: rank 0 draws the
        # shared seed from its global stream and every rank reseeds with it
        np.random.seed(int(np.random.randint(0, 2 ** 31 - 1)))
    nb = params_help.get_neighbour_matrix_by_hand(neighbour_dict_set[0], knn=2)
    net = models_att.cgcnn(F=64, mask_type="locally_connected", init_type="same", neighbour_matrix=nb,
                           in_F=2, num_layers=1, num_epochs=2, batch_size=100, dropout=0.25,
                           dir_name=os.environ["FIT_DIR_NAME"], knn=2)
    losses, _ = net.fit(tx, tl, vx, vl, output_dir=os.environ.get("FIT_JSON_DIR"))
    pred = net.predict(vx)               # restores rank 0's final checkpoint on every rank
    theta = net._net.get_params()
    np.savez(out, losses=np.asarray(losses, np.float64), theta=theta, pred=pred, rank=rank)


if __name__ == "__main__":
    main(sys.argv[1])
