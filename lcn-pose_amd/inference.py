"""inference.py of adgx/lcn-pose on the MI355X-native LCN (same CLI, inference.py:12-127).

    python inference.py --train_set h36m --test_set h36m --checkpoints best [--flip-data ...]

Test-time augmentation runs on the device: instead of concatenating the
flipped / rotated / translated copies on the host, predicting and calling
data.undo (inference.py:70-111), cgcnn.predict_tta builds the same copies
batch by batch in HBM and undoes + averages them there (same batches, same
arithmetic order; see tests/test_gpu_data.py).
"""
import argparse
import os
import pickle
import pprint

import numpy as np

from network import models_att
from tools import data, params_help

ROOT_PATH = os.path.dirname(os.path.realpath(__file__))


def parse_args():
    parser = argparse.ArgumentParser(description='inference')
    parser.add_argument('--test-indices', help='test idx ', type=str, default="1")
    parser.add_argument('--mask-type', type=str, default='locally_connected', choices=['locally_connected', 'exponential'])
    parser.add_argument('--init-type', type=str, default='same', choices=['same', 'ones', 'random'])
    parser.add_argument('--graph', help='index of graphs', type=int, default=0)
    parser.add_argument('--knn', help='expand of neighbourhood', type=int, default=2)
    parser.add_argument('--layers', help='number of layers', type=int, default=3)
    parser.add_argument('--in-joints', type=int, default=17)
    parser.add_argument('--out-joints', type=int, default=17)
    parser.add_argument('--dropout', help='dropout probability', type=float, default=0.25)
    parser.add_argument('--channels', help='number of channels', type=int, default=64)
    parser.add_argument('--subset', type=int, default=None)
    parser.add_argument('--epochs', type=int, default=200)
    parser.add_argument('--checkpoints', help='type of checkpoints', type=str, choices=['final', 'best'])
    parser.add_argument('--batch_size', help='batch size', type=int, default=200)
    parser.add_argument('--regularization', type=float, default=None)
    parser.add_argument('--learning_rate', type=float, default=0.001)
    parser.add_argument('--in-F', type=int, default=2, choices=[2, 3])
    parser.add_argument('--flip-data', action='store_true', default=False)
    parser.add_argument('--rotation-data', action='store_true', default=False)
    parser.add_argument('--translate_data', action='store_true', default=False)
    parser.add_argument("--translation_factor", type=float, default=0.1)
    parser.add_argument('--train_set', type=str, default=None, choices=["h36m", "humansc3d", "mpii"], required=True)
    parser.add_argument('--test_set', type=str, default=None, choices=["h36m", "humansc3d", "mpii"], required=True)
    try:
        return parser.parse_args()
    except SystemExit as error:
        parser.print_help()
        print(f"Error parsing arguments: {error}")
        raise


def main():
    args = parse_args()
    datareader = data.DataReader()
    gt_trainset = datareader.real_read(args.train_set, "train")
    gt_testset = datareader.real_read(args.test_set, "test")
    if args.subset is not None:
        gt_trainset = data.get_subset(gt_trainset, subset_size=args.subset, mode="camera")
        gt_testset = data.get_subset(gt_trainset, subset_size=args.subset, mode="camera")  # (sic)

    _, test_data = datareader.read_2d(gt_trainset, gt_testset)
    train_labels, test_labels = datareader.read_3d()

    translation = None
    if args.translate_data:
        if args.translation_factor < 0:
            raise ValueError("Translation factor must be non-negative")
        translation = np.random.uniform(-args.translation_factor, args.translation_factor)

    params = params_help.get_params(is_training=True, gt_dataset=train_labels)
    params_help.update_parameters(args, params)
    print(pprint.pformat(params))

    network = models_att.cgcnn(**params)
    print("Start with predictions")
    if args.flip_data or args.rotation_data or args.translate_data:
        predictions = network.predict_tta(test_data, flip=args.flip_data, rotate=args.rotation_data,
                                          translation=translation)
    else:
        predictions = network.predict(data=test_data, sess=None)
    print("Predictions done")

    result = datareader.denormalize(predictions)
    save_path = os.path.join(ROOT_PATH, 'experiment', params['dir_name'], 'result.pkl')
    if int(os.environ.get("RANK", "0")) == 0:  # one process per GPU: every rank predicted the same
        with open(save_path, 'wb') as f:
            pickle.dump(result, f)


if __name__ == '__main__':
    main()
