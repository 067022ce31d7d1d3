"""train.py of adgx/lcn-pose on the MI355X-native LCN (same CLI, train.py:12-121).

    python train.py --train_set h36m --validation_set h36m [--knn 3 --layers 3 ...]

Reads <package>/dataset/<set>_{train,val}.pkl (or $LCN_DATASET_DIR), builds the
parameters exactly as the reference (params_help.get_params + update_parameters)
and runs network.models_att.cgcnn(**params).fit(...) on liblcn.so.
"""
import argparse
import os
import pprint

import numpy as np

from network import models_att
from tools import data, params_help

ROOT_PATH = os.path.dirname(os.path.realpath(__file__))
DBG = 1


def parse_args():
    parser = argparse.ArgumentParser(description='train')
    parser.add_argument('--test-indices', help='test idx ', type=str, default="1")
    parser.add_argument('--mask-type', help='mask type', type=str, default='locally_connected',
                        choices=['locally_connected', 'exponential'])
    parser.add_argument('--init-type', help='initialization type ', type=str, default='same', choices=['same'])
    parser.add_argument('--knn', help='expand of neighbourhood', type=int, default=2)
    parser.add_argument('--layers', help='number of layers', type=int, default=3)
    parser.add_argument('--dropout', help='dropout probability', type=float, default=0)
    parser.add_argument('--channels', help='number of channels', type=int, default=64)
    parser.add_argument('--subset', help='Make a subset from the dataset passed', type=int, default=None)
    parser.add_argument('--epochs', help='number of epochs', type=int, default=25)
    parser.add_argument('--batch_size', help='batch size', type=int, default=200)
    parser.add_argument('--learning_rate', help='learning rate', type=float, default=0.001)
    parser.add_argument('--regularization', help='regularization factor', type=float, default=None)
    parser.add_argument('--in-F', help='feature channels of input data', type=int, default=2, choices=[2, 3])
    parser.add_argument('--flip-data', help='train time flip', action='store_true', default=False)
    parser.add_argument('--rotation-data', help='train time rotation', action='store_true', default=False)
    parser.add_argument('--translate_data', help='train time translate', action='store_true', default=False)
    parser.add_argument("--translation_factor", type=float, default=0.1)
    parser.add_argument("--rotation_factor", type=float, default=60)
    parser.add_argument('--resume_from', type=str, default=None)
    parser.add_argument('--output_file', type=str, default=None)
    parser.add_argument('--train_set', type=str, default=None, choices=["h36m", "humansc3d", "mpii"], required=True)
    parser.add_argument('--validation_set', type=str, default=None, choices=["h36m", "humansc3d", "mpii"], required=True)
    parser.add_argument('--test_set', type=str, default=None, choices=["h36m", "humansc3d", "mpii"])
    parser.add_argument('--n_test', help='number of test for random search', type=int, default=1)
    try:
        return parser.parse_args()
    except SystemExit:
        parser.print_help()
        raise


def main():
    args = parse_args()
    datareader = data.DataReader()
    gt_trainset = datareader.real_read(args.train_set, "train")
    gt_valset = datareader.real_read(args.validation_set, "val")
    if DBG:
        if args.rotation_data:
            gt_trainset.extend(datareader.real_read(args.train_set, "train_rotated"))
        if args.translate_data:
            gt_trainset.extend(datareader.real_read(args.train_set, "train_translation"))
    if args.subset is not None:
        gt_trainset = data.get_subset(gt_trainset, subset_size=args.subset, mode="camera")
        gt_valset = data.get_subset(gt_valset, subset_size=args.subset, mode="camera")

    train_data, val_data = datareader.read_2d(gt_trainset, gt_valset)
    train_labels, val_labels = datareader.read_3d()
    dataset_copy, labelset_copy = train_data.copy(), train_labels.copy()
    if args.flip_data:
        train_data = np.concatenate((train_data, data.flip_data(dataset_copy)), axis=0)
        train_labels = np.concatenate((train_labels, data.flip_data(labelset_copy)), axis=0)
    if DBG == 0:  # (the reference's disabled train-time translation / rotation)
        pass

    params = params_help.get_params(is_training=True, gt_dataset=train_labels)
    params_help.update_parameters(args, params)
    print(pprint.pformat(params))

    network = models_att.cgcnn(**params)
    try:
        losses, t_step = network.fit(train_data, train_labels, val_data, val_labels, args.output_file,
                                     starting_checkpoint=args.resume_from)
        print(losses)
        print(t_step)
    except KeyboardInterrupt:
        print('Training interrupted')
    except Exception as e:
        print('Error during training: ', e)
        raise SystemExit


if __name__ == '__main__':
    main()
