"""CPU restatement of the reference's evaluation path -- TEST INFRASTRUCTURE
ONLY (tests/, bench.py's cpu_baseline leg and smoke() may import it; the
product never does).

Follows, line by line and in numpy float64 like the reference:
  * image_to_camera_frame   tools/tools.py:183-194
  * procrustes              tools/tools.py:96-181 (scaling=True, reflection='best')
  * align_to_gt             tools/tools.py:197-202
  * _eval's per-frame loop  evaluate.py:53-73 (error_per_joint, best frame)
  * _eval's aggregation     evaluate.py:75-110 (per action + PCK@50 mm, or per joint)

Pinned by tests/golden/ref_eval.npz: outputs of the reference's own
tools.tools functions on seeded synthetic frames (oracle/gen_golden.py).
"""
from __future__ import annotations

import numpy as np

THRESHOLD = 50  # mm, evaluate.py:10


def image_to_camera_frame(pose3d_image_frame, box, camera, root_depth):
    """tools.py:183-194; camera = (cx, cy, fx, fy)."""
    ratio = (box[2] - box[0] + 1) / 2000.0
    p = pose3d_image_frame.copy()
    p[:, 2] = p[:, 2] / ratio + root_depth
    cx, cy, fx, fy = camera
    p[:, 0] = (p[:, 0] - cx) / fx
    p[:, 1] = (p[:, 1] - cy) / fy
    p[:, 0] *= p[:, 2]
    p[:, 1] *= p[:, 2]
    return p


def procrustes(A, B):
    """tools.py:96-181 with scaling=True, reflection='best': returns Z."""
    A_bar, B_bar = A.mean(0), B.mean(0)
    A0, B0 = A - A_bar, B - B_bar
    A_norm, B_norm = np.sqrt((A0 ** 2).sum()), np.sqrt((B0 ** 2).sum())
    A0 = A0 / A_norm
    B0 = B0 / B_norm
    U, s, Vt = np.linalg.svd(A0.T.dot(B0))
    R = Vt.T.dot(U.T)
    return A_norm * s.sum() * B0.dot(R) + A_bar


def frame_errors(pred, gt, box, cam, root_depth, protocol2):
    """evaluate.py:53-61 for every frame: err [N, 17]."""
    n = pred.shape[0]
    err = np.empty((n, 17))
    for i in range(n):
        p = image_to_camera_frame(pred[i], box[i], cam[i], root_depth[i])
        if protocol2:
            p = procrustes(gt[i], p)
        err[i] = np.sqrt(np.square(p - gt[i]).sum(axis=1))
    return err


def best_frame(err):
    """evaluate.py:63-68: first frame with the smallest mean joint error."""
    m = err.mean(axis=1)
    idx = int(np.argmin(m))
    return idx, float(m[idx])


def aggregate(results, actions, range_action, per_joint):
    """evaluate.py:75-110 on results [N, 17]: (final_result, final_results_pck)."""
    final_pck = []
    if not per_joint:
        final_result = []
        index = {a: [] for a in range_action}
        for i, a in enumerate(actions):
            index[a].append(i)
        for a in range_action:
            final_result.append(np.mean(results[index[a]]))
            arr = np.array(results[index[a]])
            if len(arr < THRESHOLD) == 0:
                final_pck.append(0)
            else:
                final_pck.append((len(arr[arr < THRESHOLD]) / (len(arr) * arr.shape[1])) * 100)
        error = np.mean(np.array(final_result))
        final_result.append(error)
        final_pck.append(np.mean(np.array(final_pck)))
    else:
        error = np.mean(results, axis=0)
        final_result = error.tolist() + [np.mean(error)]
        final_pck.append((len(results[results < THRESHOLD]) / (len(results) * results.shape[1])) * 100)
    return final_result, final_pck
