"""Generate the golden fixtures under tests/golden/ -- TEST INFRASTRUCTURE ONLY.

Run in the build container (it reads /root/reference, which does not exist on
the GPU box):  ``python oracle/gen_golden.py``.

What it pins, and from where:

* ``ref_helpers.npz`` -- outputs of the reference's OWN numpy helpers, imported
  from /root/reference:
    - ``tools.params_help.get_neighbour_matrix_by_hand(neighbour_dict_set[0], knn)``
      for knn = 1..5 (params_help.py:8-20, filter_hub.py:4-24);
    - ``network.models_att.get_exponential_matrix()`` (models_att.py:14-69),
      imported with an empty ``tensorflow`` placeholder module because the
      module does ``import tensorflow as tf`` at top level and TF is not
      installed (the function itself is pure numpy);
    - ``tools.data.flip_data / rotate_data / translation_data / undo`` on
      seeded inputs (data.py:10-25, 289-322, 27-54, 269-287), imported with an ``h5py``
      placeholder (data.py:3 imports it and never uses it).
* ``ref_datareader.npz`` -- the reference's ``tools.data.DataReader``
  (read_2d / read_3d / denormalize, data.py:338-489) on synthetic in-memory
  items (``synthetic_gt``; float64 and float32 joints).
* ``ref_eval.npz`` -- evaluate.py's per-frame errors (protocol 1 and 2) from
  the reference's ``tools.tools.image_to_camera_frame`` / ``align_to_gt``
  (tools.py:96-202) on synthetic frames (``synthetic_frames``).
* ``notebook_masks.npz`` -- the neighbour matrices printed by the reference's
  own Kaggle runs (parameter dumps in kaggle/custom-dataset-h36m.ipynb, knn=2,
  and kaggle/custom-dataset-humansc3d.ipynb, knn=1).
* ``notebook_facts.json`` -- the learning rates and step arithmetic printed in
  those logs (lr at step 7798 and 957; total steps 1 559 752 and 95 746).
* ``oracle_*.npz`` -- float64 oracle forward/gradient/Adam vectors at small
  sizes (regression pins for the oracle itself; the TF graph arithmetic is
  unpinned, see oracle/lcn_oracle.py).
"""
from __future__ import annotations

import json
import os
import re
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, HERE)
import lcn_oracle as O  # noqa: E402


def _import_reference():
    sys.modules.setdefault("h5py", types.ModuleType("h5py"))
    sys.modules.setdefault("tensorflow", types.ModuleType("tensorflow"))
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(REF, "tools"))
    sys.path.insert(0, os.path.join(REF, "network"))
    import params_help, filter_hub, data  # noqa
    import models_att  # noqa
    return params_help, filter_hub, data, models_att


def ref_helpers():
    params_help, filter_hub, data, models_att = _import_reference()
    out = {}
    for knn in range(1, 6):
        out[f"neighbour_knn{knn}"] = params_help.get_neighbour_matrix_by_hand(
            filter_hub.neighbour_dict_set[0], knn=knn)
    import contextlib, io
    with contextlib.redirect_stdout(io.StringIO()):
        out["exp_matrix"] = models_att.get_exponential_matrix()
    rng = np.random.default_rng(7)
    x2 = rng.uniform(-1, 1, size=(5, 34))
    x3 = rng.uniform(-1, 1, size=(5, 51))
    out["flip_in2"], out["flip_out2"] = x2, data.flip_data(x2)
    out["flip_in3"], out["flip_out3"] = x3, data.flip_data(x3)
    out["rot_in2"], out["rot_out2"] = x2, data.rotate_data(x2, 180)
    out["rot_in3"], out["rot_out3"] = x3, data.rotate_data(x3, 180)
    out["rot_out3_90"] = data.rotate_data(x3, 90)
    preds = rng.uniform(-1, 1, size=(4 * 5, 51))
    # appended after the draws above so the earlier vectors keep their values
    rng2 = np.random.default_rng(11)
    t2 = rng2.uniform(-1, 1, size=(6, 34))
    t3 = rng2.uniform(-1, 1, size=(6, 51))
    out["trans_in2"], out["trans_out2"] = t2, data.translation_data(t2, 0.07)
    out["trans_in3"], out["trans_out3"] = t3, data.translation_data(t3, -0.03)
    out["rot_out2_37"] = data.rotate_data(t2, 37.0)
    out["undo_in"] = preds
    out["undo_out_fr"] = data.undo(preds[:15], {"f": 1, "r": 2}, number_actions=2)
    out["undo_out_frt"] = data.undo(preds, {"f": 1, "r": 2, "t": 3}, number_actions=3,
                                    translation=0.05)
    return out


def synthetic_gt(n, seed, dtype):
    """In-memory dataset items with the reference's per-frame dict schema
    (gendb*.py): joint_3d_image [17, 3] (pixels, depth), camera_param.name,
    cameraid / videoid / subject / action."""
    rng = np.random.default_rng(seed)
    cams = ["54138969", "55011271", "58860488", "60457274", "cam_3", "17", "65906101"]
    items = []
    for i in range(n):
        cam = cams[i % len(cams)]
        j = np.concatenate([rng.uniform(0, 1000, (17, 2)), rng.uniform(-300, 300, (17, 1))], 1)
        items.append({"joint_3d_image": j.astype(dtype), "camera_param": {"name": cam},
                      "cameraid": cam, "videoid": i // 3, "subject": f"S{i % 3}",
                      "action": f"a{i % 4}"})
    return items


def data_reader():
    """tools.data.DataReader read_2d / read_3d / denormalize of the reference
    on synthetic items (float64 and float32 joints)."""
    _, _, data, _ = _import_reference()
    out = {}
    for tag, dt in (("f64", np.float64), ("f32", np.float32)):
        tr, te = synthetic_gt(23, 1, dt), synthetic_gt(15, 2, dt)
        r = data.DataReader()
        x_tr, x_te = r.read_2d(tr, te)
        y_tr, y_te = r.read_3d()
        pred = np.random.default_rng(3).uniform(-1, 1, (15, 51))
        res = r.denormalize(pred)
        out[f"{tag}_x_train"], out[f"{tag}_x_test"] = x_tr, x_te
        out[f"{tag}_y_train"], out[f"{tag}_y_test"] = y_tr, y_te
        out[f"{tag}_pred"] = pred
        out[f"{tag}_denorm"] = np.stack([d["result"] for d in res])
        out[f"{tag}_denorm_keys"] = np.array([f"{d['cameraid']}|{d['videoid']}|{d['subject']}|{d['action']}"
                                              for d in res])
    return out


def synthetic_frames(n, seed):
    """Camera-space ground truth and image-frame predictions with the schema
    evaluate.py reads (joint_3d_camera, box, camera_param cx/cy/fx/fy,
    root_depth): predictions are the ground truth projected the way
    image_to_camera_frame inverts it, then rotated, scaled and perturbed."""
    rng = np.random.default_rng(seed)
    root = np.stack([rng.uniform(-500, 500, n), rng.uniform(-300, 300, n), rng.uniform(3500, 6500, n)], 1)
    gt = root[:, None, :] + rng.uniform(-800, 800, (n, 17, 3))
    gt[:, 0] = root
    box = np.stack([rng.uniform(0, 400, n), rng.uniform(0, 400, n)], 1)
    box = np.concatenate([box, box + rng.uniform(200, 900, (n, 1))], 1)
    cam = np.stack([rng.uniform(480, 520, n), rng.uniform(480, 520, n),
                    rng.uniform(1100, 1200, n), rng.uniform(1100, 1200, n)], 1)
    ang = rng.uniform(-0.3, 0.3, n)
    c, s_ = np.cos(ang), np.sin(ang)
    pert = gt.copy()
    x0 = pert[..., 0] - root[:, None, 0]
    z0 = pert[..., 2] - root[:, None, 2]
    pert[..., 0] = root[:, None, 0] + c[:, None] * x0 - s_[:, None] * z0
    pert[..., 2] = root[:, None, 2] + s_[:, None] * x0 + c[:, None] * z0
    pert = root[:, None, :] + (pert - root[:, None, :]) * rng.uniform(0.9, 1.1, (n, 1, 1))
    pert += rng.normal(0, 20, pert.shape)
    ratio = (box[:, 2] - box[:, 0] + 1) / 2000.0
    pred = np.empty_like(pert)
    pred[..., 0] = pert[..., 0] / pert[..., 2] * cam[:, None, 2] + cam[:, None, 0]
    pred[..., 1] = pert[..., 1] / pert[..., 2] * cam[:, None, 3] + cam[:, None, 1]
    pred[..., 2] = (pert[..., 2] - root[:, None, 2]) * ratio[:, None]
    return pred, gt, box, cam, root[:, 2].copy()


def ref_eval():
    """Per-frame evaluation of the reference (evaluate.py:53-61) with its own
    tools.tools.image_to_camera_frame / align_to_gt (tools.py:96-202) on
    synthetic frames; matplotlib is imported by tools.py for plotting only."""
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(REF, "tools"))
    import tools as ref_tools  # noqa
    pred, gt, box, cam, rd = synthetic_frames(257, seed=21)
    out = {"pred": pred, "gt": gt, "box": box, "cam": cam, "root_depth": rd}
    for proto in (1, 2):
        err = np.empty((len(pred), 17))
        cam_pose = np.empty_like(pred)
        for i in range(len(pred)):
            camera = {"cx": cam[i, 0], "cy": cam[i, 1], "fx": cam[i, 2], "fy": cam[i, 3]}
            p = ref_tools.image_to_camera_frame(pose3d_image_frame=pred[i], box=box[i], camera=camera,
                                                rootIdx=0, root_depth=rd[i])
            if proto == 1:
                cam_pose[i] = p
            else:
                p = ref_tools.align_to_gt(pose=p, pose_gt=gt[i])
                cam_pose[i] = p
            err[i] = np.sqrt(np.square(p - gt[i]).sum(axis=1))
        out[f"p{proto}_pose"] = cam_pose
        out[f"p{proto}_err"] = err
    return out


def notebook_masks():
    res = {}
    for fname, key in (("custom-dataset-h36m.ipynb", "nb_h36m_knn2"),
                       ("custom-dataset-humansc3d.ipynb", "nb_humansc3d_knn1")):
        nb = json.load(open(os.path.join(REF, "kaggle", fname)))
        for cell in nb["cells"]:
            txt = "".join("".join(o.get("text", [])) for o in cell.get("outputs", []))
            k = txt.find("'neighbour_matrix': array(")
            if k < 0:
                continue
            body = txt[k + len("'neighbour_matrix': array("):]
            body = body[:body.index("dtype=float32)")]
            nums = [float(v) for v in re.findall(r"[01]\.", body)]
            res[key] = np.array(nums, np.float32).reshape(17, 17)
            break
    return res


def notebook_facts():
    facts = {}
    nb = json.load(open(os.path.join(REF, "kaggle", "custom-dataset-h36m.ipynb")))
    txt = "".join("".join(o.get("text", [])) for c in nb["cells"] for o in c.get("outputs", []))
    m = re.search(r"Total steps to be done to complete all the epochs: (\d+)", txt)
    facts["h36m_total_steps"] = int(m.group(1))
    m = re.search(r"step (\d+) / \d+ \(epoch 1\.00 / 200\):\s+learning_rate = ([0-9.e+-]+)", txt)
    facts["h36m_step1"], facts["h36m_lr1"] = int(m.group(1)), float(m.group(2))
    facts["h36m_batch"], facts["h36m_epochs"] = 200, 200
    nb = json.load(open(os.path.join(REF, "kaggle", "custom-dataset-humansc3d.ipynb")))
    txt = "".join("".join(o.get("text", [])) for c in nb["cells"] for o in c.get("outputs", []))
    m = re.search(r"Total steps to be done to complete all the epochs: (\d+)", txt)
    facts["sc3d_total_steps"] = int(m.group(1))
    m = re.search(r"step (\d+) / \d+ \(epoch 1\.00 / 100\):\s+learning_rate = ([0-9.e+-]+)", txt)
    facts["sc3d_step1"], facts["sc3d_lr1"] = int(m.group(1)), float(m.group(2))
    facts["sc3d_batch"], facts["sc3d_epochs"] = 512, 100
    return facts


def oracle_vectors():
    """float64 oracle outputs for a few small configurations."""
    cases = {
        "lc_knn3_F8_L2_B24": dict(F=8, L=2, knn=3, B=24, mask="locally_connected", in_F=2),
        "lc_knn1_F8_L1_B16_in3": dict(F=8, L=1, knn=1, B=16, mask="locally_connected", in_F=3),
        "exp_F8_L1_B16": dict(F=8, L=1, knn=2, B=16, mask="exponential", in_F=2),
        "lc_knn3_F64_L3_B32": dict(F=64, L=3, knn=3, B=32, mask="locally_connected", in_F=2),
    }
    res = {}
    for name, c in cases.items():
        cfg = O.Config(F=c["F"], in_F=c["in_F"], num_layers=c["L"], mask_type=c["mask"],
                       neighbour=O.neighbour_matrix(c["knn"]))
        params = O.init_params(cfg, seed=1)
        rng = np.random.default_rng(2)
        x = rng.uniform(-1, 1, size=(c["B"], 17 * c["in_F"])).astype(np.float32)
        lab = rng.uniform(-1, 1, size=(c["B"], 51)).astype(np.float32)
        out, cache = O.forward(cfg, params, x, np.float64)
        grads = O.backward(cfg, params, cache, lab, np.float64)
        d = {"x": x, "lab": lab, "out": out, "loss": np.float64(O.mse_loss(out, lab)),
             "params_flat": O.flatten(cfg, params)}
        d["grads_flat"] = np.concatenate([grads[n].ravel() for n, _ in O.param_specs(cfg)])
        p2 = {k: v.copy() for k, v in params.items()}
        st = O.adam_init(cfg, p2)
        O.adam_step(cfg, p2, {k: v.astype(np.float32) for k, v in grads.items()}, st)
        d["params_after_adam"] = O.flatten(cfg, p2)
        if c["F"] > 16:
            # full vectors would be tens of MB: keep per-tensor norms and a
            # seeded sample of entries (params are re-created from seed=1)
            sel = np.random.default_rng(3).choice(d["grads_flat"].size, 4096, replace=False)
            d["sample_idx"] = sel
            for k in ("grads_flat", "params_after_adam", "params_flat"):
                d[k + "_sample"] = d.pop(k)[sel]
            d["grad_norms"] = np.array([np.linalg.norm(grads[n]) for n, _ in O.param_specs(cfg)])
        d["meta"] = np.array(json.dumps(c))
        res[name] = d
    return res


def main():
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, "ref_helpers.npz"), **ref_helpers())
    np.savez(os.path.join(OUT, "notebook_masks.npz"), **notebook_masks())
    np.savez(os.path.join(OUT, "ref_datareader.npz"), **data_reader())
    np.savez_compressed(os.path.join(OUT, "ref_eval.npz"), **ref_eval())
    with open(os.path.join(OUT, "notebook_facts.json"), "w") as f:
        json.dump(notebook_facts(), f, indent=1)
    for name, d in oracle_vectors().items():
        np.savez_compressed(os.path.join(OUT, f"oracle_{name}.npz"), **d)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
