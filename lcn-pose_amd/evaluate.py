"""evaluate.py of adgx/lcn-pose with the per-frame loop on the MI355X
(same CLI and outputs, evaluate.py:11-200).

    python evaluate.py --filename h36m --test-indices 1,2 [--per-joint] [--protocol2]

The reference walks the test set one frame at a time in Python:
image_to_camera_frame, optional Procrustes alignment (a numpy SVD per frame),
per-joint error (evaluate.py:53-73).  Here all frames go to the device in one
lcn_eval_mpjpe launch (lcn_amd.native.eval_mpjpe, kernels_eval.hip); the
aggregation per action / per joint and PCK@50 mm stay numpy on the host
(evaluate.py:75-110, ``aggregate``), as do the log tables and best-frame files.
"""
from __future__ import annotations

import argparse
import os
import pickle
import time

import numpy as np

from lcn_amd.native import eval_mpjpe

ROOT_PATH = os.path.dirname(os.path.realpath(__file__))
THRESHOLD = 50  # mm


def parse_args():
    parser = argparse.ArgumentParser(description='evaluate')
    parser.add_argument('--protocol2', help='whether use Procrustes', action='store_true')
    parser.add_argument('--test-indices', help='test idx list to eval', required=True, type=str)
    parser.add_argument('--per-joint', help='joint-wise evaluation', action='store_true')
    parser.add_argument('--filename', type=str, default=None, help='Filename of the dataset',
                        choices=["h36m", "humansc3d", "mpii"], required=True)
    try:
        args = parser.parse_args()
    except SystemExit:
        parser.print_help()
        raise
    return args


def frame_arrays(dataitem_gt):
    """gt [N,17,3], box [N,4], cam [N,4] (cx, cy, fx, fy), root_depth [N] from
    the dataset items evaluate.py reads (evaluate.py:54-57)."""
    n = len(dataitem_gt)
    gt = np.empty((n, 17, 3))
    box = np.empty((n, 4))
    cam = np.empty((n, 4))
    rd = np.empty(n)
    for i, it in enumerate(dataitem_gt):
        gt[i] = it['joint_3d_camera']
        box[i] = np.asarray(it['box'], dtype=np.float64)[:4]
        c = it['camera_param']
        cam[i] = (c['cx'], c['cy'], c['fx'], c['fy'])
        rd[i] = it['root_depth']
    return gt, box, cam, rd


def frame_errors(preds, dataitem_gt, protocol2, device=0):
    """error_per_joint of every frame (evaluate.py:53-61): [N, 17] float64."""
    gt, box, cam, rd = frame_arrays(dataitem_gt)
    return eval_mpjpe(np.asarray(preds, dtype=np.float64).reshape(-1, 17, 3), gt, box, cam, rd,
                      protocol2=protocol2, device=device)


def aggregate(results, actions, range_action, per_joint):
    """evaluate.py:75-110: per action mean error and PCK@50 mm (+ averages),
    or per joint mean error (+ average) and one PCK.  Same numpy reductions
    over the same row order as the reference's index lists."""
    final_results_pck = []
    if not per_joint:
        actions = np.asarray(actions)
        final_result = []
        for a in range_action:
            arr = results[actions == a]
            final_result.append(np.mean(arr))
            if len(arr < THRESHOLD) == 0:
                final_results_pck.append(0)
            else:
                final_results_pck.append((len(arr[arr < THRESHOLD]) / (len(arr) * arr.shape[1])) * 100)
        error = np.mean(np.array(final_result))
        final_result.append(error)
        final_results_pck.append(np.mean(np.array(final_results_pck)))
    else:
        error = np.mean(results, axis=0)
        final_result = error.tolist() + [np.mean(error)]
        final_results_pck.append((len(results[results < THRESHOLD]) / (len(results) * results.shape[1])) * 100)
    return final_result, final_results_pck


def _eval(test_name, dataitem_gt, commd, range_action):
    """evaluate.py:29-110."""
    result_path = os.path.join(ROOT_PATH, 'experiment', test_name, 'result.pkl')
    with open(result_path, 'rb') as f:  # written by inference.py
        preds = [res_item['result'] for res_item in pickle.load(f)]
    preds = np.reshape(preds, (-1, 17, 3))
    if len(preds) > len(dataitem_gt):
        preds = preds[:len(dataitem_gt)]
    assert len(preds) == len(dataitem_gt)
    results = frame_errors(preds, dataitem_gt, 'protocol2' in commd)
    mean = results.mean(axis=1)
    best_frame_idx = int(np.argmin(mean))  # first frame with the smallest mean error (:63-68)
    error_best_frame = float(mean[best_frame_idx])
    for idx in range(0, len(results), 10000):
        print('step:%d' % idx + '-' * 20)
        print(np.mean(results[idx]))
    if 'action' in commd:
        actions = [d['action'] for d in dataitem_gt]
        final_result, final_pck = aggregate(results, actions, range_action, per_joint=False)
    elif 'joint' in commd:
        final_result, final_pck = aggregate(results, None, range_action, per_joint=True)
    else:
        assert 0, 'not implemented commd'
    # the reference also returns the best frame's camera-space pose, which its
    # caller only writes to a file it then overwrites (:170-177)
    return final_result, final_pck, best_frame_idx, error_best_frame, dataitem_gt[best_frame_idx]


def _table(field_names, rows):
    widths = [max(len(str(f)), *(len(str(r[i])) for r in rows)) for i, f in enumerate(field_names)]
    sep = '+' + '+'.join('-' * (w + 2) for w in widths) + '+'
    line = lambda vals: '|' + '|'.join(' %s ' % str(v).center(w) for v, w in zip(vals, widths)) + '|'
    return '\n'.join([sep, line(field_names), sep] + [line(r) for r in rows] + [sep])


def eval(commd, test_indices, pkl=""):
    err_dict = {}
    print('loading dataset')
    base = os.environ.get("LCN_DATASET_DIR", os.path.join(ROOT_PATH, "dataset"))  # as tools/data.py
    with open(os.path.join(base, pkl + "_test.pkl"), 'rb') as f:
        dataitem_gt = pickle.load(f)
    range_action = list({item["action"] for item in dataitem_gt})
    fields = (['test_name'] + range_action + ['avg']) if 'action' in commd else \
        (['test_name'] + list(range(0, 17)) + ['avg'])
    for i in test_indices:
        test_name = 'test%d' % i
        err_dict[test_name], pck, best_idx, best_err, best_gt = _eval(test_name, dataitem_gt, commd,
                                                                     range_action)
        rows = [[test_name] + ['%.2f' % d for d in err_dict[test_name]]]
        if 'action' in commd:
            rows.append([test_name + " - PCK" + str(THRESHOLD)] + ['%.2f' % d for d in pck])
        time_str = time.strftime('%Y-%m-%d-%H-%M')
        exp = os.path.join(ROOT_PATH, 'experiment', "test" + str(i))
        with open(os.path.join(exp, 'err_{}_{}.log'.format(commd, time_str)), 'w') as f:
            print(_table(fields, rows), file=f)
        if 'action' in commd:
            print("Printing PCK Table")
            print(_table(fields, rows))
        # evaluate.py:170-183 writes both pickles to the same path (sic): the
        # ground-truth item is what remains
        with open(os.path.join(exp, 'best_frame_predicted_{}_{}.pkl'.format(commd, time_str)), 'wb') as f:
            pickle.dump(best_gt, f)
        with open(os.path.join(exp, 'best_frame_{}_{}.txt'.format(commd, time_str)), 'w') as f:
            f.write('best frame idx: %d\n' % best_idx)
            f.write('best frame error: %.2f\n' % best_err)
    if 'action' not in commd:
        print("Printing MPJPE Table")
        print(_table(fields, [[k] + ['%.2f' % d for d in v] for k, v in err_dict.items()]))
    return err_dict


if __name__ == '__main__':
    args = parse_args()
    test_indices = sorted([int(i) for i in args.test_indices.split(',')])
    commd = '_joint' if args.per_joint else '_action'
    if args.protocol2:
        commd += '_protocol2'
    print('=> commd:', commd)
    print('=> eval experiments:', test_indices)
    eval(commd=commd, test_indices=test_indices, pkl=args.filename)
