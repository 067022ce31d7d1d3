"""Step time of fit's loop at the reference's own batch sizes (200: H36M,
512: HumanSC3D), dataset resident in HBM, one lcn_train_step_indexed per
step as cgcnn.fit runs it (host permutation indices, loss read back)."""
import os
import sys
import time

import numpy as np

R = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "lcn-pose_amd"))
from lcn_amd import native  # noqa: E402
from lcn_amd.init import init_flat  # noqa: E402
from tools.params_help import get_neighbour_matrix_by_hand  # noqa: E402
from tools.filter_hub import neighbour_dict_set  # noqa: E402

CASES = ((2, 200), (1, 512), (3, 1024), (3, 2048), (3, 4096))
if os.environ.get("SMALL_CASES"):  # e.g. "2:200,1:512"
    CASES = tuple(tuple(int(v) for v in c.split(":")) for c in os.environ["SMALL_CASES"].split(","))
for knn, B in CASES:
    nb = get_neighbour_matrix_by_hand(neighbour_dict_set[0], knn=knn)
    net = native.Network(F=64, in_F=2, num_layers=3, mask_type="locally_connected",
                         mask_matrix=(nb.T != 0).astype(np.float32), max_batch=B, device=0)
    net.set_params(init_flat(net.param_layout(), net.n_params, nb, seed=0))
    N = 100000
    rng = np.random.default_rng(0)
    net.dataset_upload(0, rng.uniform(-1, 1, (N, 34)))
    net.dataset_upload(1, rng.uniform(-1, 1, (N, 51)))
    perm = rng.permutation(N)
    for i in range(20):
        net.train_step_indexed(0, 1, perm[i * B:(i + 1) * B])
    n = 300
    t0 = time.perf_counter()
    for i in range(n):
        j = (i * B) % (N - B)
        loss, lr = net.train_step_indexed(0, 1, perm[j:j + B])
    dt = (time.perf_counter() - t0) / n
    print(f"knn {knn} B {B}: {dt * 1e3:.3f} ms/step, {B / dt:,.0f} poses/s", flush=True)
    net.close()
