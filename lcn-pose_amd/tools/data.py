"""Dataset reading, normalisation and the augmentation helpers of the CLIs.

Host-side numpy, behaviour of the reference's tools/data.py (vectorised; the
same floating-point operations in the same order, so the arrays are
bit-identical):

  flip_data           :10-25     translation_data   :27-54
  get_subset*         :56-201    untranslation_data :205-218
  unflip_data         :236-249   undo               :269-287
  rotate_data         :289-322   DataReader         :324-489

Pickled datasets are read from ``<package>/dataset/<name>_<split>.pkl`` as the
reference does, or from ``$LCN_DATASET_DIR`` when set.  The augmentation
helpers are the host path; the device path of inference's test-time
augmentation is cgcnn.predict_tta (lcn_amd.tta + liblcn).
"""
from __future__ import annotations

import os
import pickle

import numpy as np

ROOT_PATH = os.path.join(os.path.dirname(os.path.realpath(__file__)), "..")
LEFT = [4, 5, 6, 11, 12, 13]
RIGHT = [1, 2, 3, 14, 15, 16]


def flip_data(data):
    flipped = data.copy().reshape((len(data), 17, -1))
    flipped[:, :, 0] *= -1
    flipped[:, LEFT + RIGHT] = flipped[:, RIGHT + LEFT]
    return flipped.reshape(data.shape)


def translation_data(data, translation_factor=0.5):
    if isinstance(translation_factor, np.ndarray):
        # the reference's per-item branch (:39-45) adds the whole array to one
        # element and fails; only the scalar factor is usable
        raise ValueError("setting an array element with a sequence")
    d = data.copy().reshape((len(data), 17, -1))
    d[:, :, 0] += translation_factor
    d[:, :, 1] += translation_factor
    if d.shape[2] == 3:
        d[:, :, 2] += translation_factor
    return d.reshape(data.shape)


def untranslation_data(data, translation_factor=0.5):
    d = data.copy().reshape((-1, 17, 3))
    d -= translation_factor
    return d.reshape(data.shape)


def unflip_data(data):
    d = data.copy().reshape(-1, 17, 3)
    d[:, :, 0] *= -1
    d[:, LEFT + RIGHT] = d[:, RIGHT + LEFT]
    return d


def rotate_data(data, angle=180):
    theta = np.radians(angle)
    Rz = np.array([[np.cos(theta), -np.sin(theta), 0],
                   [np.sin(theta), np.cos(theta), 0],
                   [0, 0, 1]])
    r = data.copy().reshape((len(data), 17, -1))
    k = r.shape[2]
    if k == 2:
        piv = r[:, 0:1, :2].copy()
        r = (r - piv) @ Rz.T[:2, :2] + piv
    elif k == 3:
        piv = r[:, 0:1, :3].copy()
        r[:, :, :3] = (r[:, :, :3] - piv) @ Rz.T + piv
    return r.reshape(data.shape)


def undo(data, op_ord, number_actions=2, angle=180, translation=0.5):
    d = data.copy().reshape(number_actions + 1, -1, 17, 3)
    if "f" in op_ord:
        d[op_ord["f"]] = unflip_data(d[op_ord["f"]])
    if "r" in op_ord:
        d[op_ord["r"]] = rotate_data(d[op_ord["r"]], angle)
    if "t" in op_ord:
        d[op_ord["t"]] = untranslation_data(d[op_ord["t"]], translation)
    return np.mean(d, axis=0).reshape((-1, 17 * 3))


def _subset_by(gt_dataset, key, subset_size):
    if not all(key in item for item in gt_dataset):
        raise ValueError(f"The dataset must contain '{key}' key in each item.")
    names = set(item[key] for item in gt_dataset)
    subsets = {n: [] for n in names}
    for item in gt_dataset:
        value = np.random.uniform(0, 1)  # drawn per item, as the reference
        if len(subsets[item[key]]) < subset_size // len(names) and value:
            subsets[item[key]].append(item)
    return [it for s in subsets.values() for it in s]


def get_subset(gt_dataset, subset_size=1000, mode="camera"):
    """The reference's CLIs call this with mode="camera" (train.py:74-75)."""
    if subset_size is None:
        return gt_dataset
    keys = {"camera": "cameraid", "action": "action", "subject": "subject"}
    if mode not in keys:
        raise NotImplementedError(f"subset mode {mode!r}")
    return _subset_by(gt_dataset, keys[mode], subset_size)


def camera_resolution(name) -> tuple:
    """(res_w, res_h) of a camera (data.py:355-366)."""
    name = str(name)
    if name in ("54138969", "60457274"):
        return 1000, 1002
    if name in ("55011271", "58860488", "50591643", "65906101"):
        return 1000, 1000
    if name.find("cam_") != -1:
        return 2048, 2048
    if int(name) >= 0:
        return 2048, 2048
    raise AssertionError("invalid camera name %s" % name)


def _groups(items):
    """indices of the items per camera resolution (res_w, res_h as Python ints,
    so numpy keeps the operand dtype exactly as the reference's per-item
    arithmetic does)."""
    res = [camera_resolution(it["camera_param"]["name"]) for it in items]
    out = {}
    for i, r in enumerate(res):
        out.setdefault(r, []).append(i)
    return {r: np.array(ix) for r, ix in out.items()}


class DataReader(object):
    def __init__(self):
        self.gt_trainset = None
        self.gt_testset = None
        self.dt_dataset = None

    def real_read(self, subset, type):
        file_name = "%s_%s.pkl" % (subset, type)
        print("loading %s" % file_name)
        base = os.environ.get("LCN_DATASET_DIR", os.path.join(ROOT_PATH, "dataset"))
        with open(os.path.join(base, file_name), "rb") as f:
            return pickle.load(f)

    def read_2d(self, gt_trainset, gt_testset, which="scale"):
        if self.gt_trainset is None:
            self.gt_trainset = gt_trainset
        if self.gt_testset is None:
            self.gt_testset = gt_testset
        if which != "scale":
            raise AssertionError("not support normalize type %s" % which)

        def norm(items):
            arr = np.empty((len(items), 17, 2))  # float64, as data.py:344-345
            for i, it in enumerate(items):
                arr[i] = it["joint_3d_image"][:, :2]
            for (w, h), ix in _groups(items).items():
                arr[ix] = arr[ix] / w * 2 - [1, h / w]  # data.py:367, 382
            return arr.reshape((len(arr), -1))

        return norm(self.gt_trainset), norm(self.gt_testset)

    def read_3d(self, which="scale"):
        if which != "scale":
            raise AssertionError("not support normalize type %s" % which)

        def lab(items):
            out = np.empty((len(items), 17, 3))
            for (w, h), ix in _groups(items).items():
                # the item's own dtype, then stored as float64 (data.py:416-418)
                j = np.stack([items[i]["joint_3d_image"] for i in ix])
                out[ix, :, :2] = j[:, :, :2] / w * 2 - [1, h / w]
                out[ix, :, 2:] = j[:, :, 2:] / w * 2
            return out.reshape((-1, 17 * 3))

        return lab(self.gt_trainset), lab(self.gt_testset)

    def denormalize(self, data, which="scale"):
        if which != "scale":
            raise AssertionError
        data = data.reshape((-1, 17, 3)).copy()
        items = self.gt_testset
        for (w, h), ix in _groups(items).items():
            data[ix, :, :2] = (data[ix, :, :2] + [1, h / w]) * w / 2  # data.py:466-467
            data[ix, :, 2:] = data[ix, :, 2:] * w / 2
        return [{"cameraid": it["cameraid"], "videoid": it["videoid"], "subject": it["subject"],
                 "action": it["action"], "result": data[i]} for i, it in enumerate(items)]
