"""Inference CLI of the MI355X-native LCN; takes the flags of the reference's
inference.py (inference.py:16-40; schema in tools/cli_flags.py).

    python inference.py --train_set h36m --test_set h36m --checkpoints best [--flip-data ...]

Test-time augmentation runs on the device: instead of concatenating the
flipped / rotated / translated copies on the host, predicting and calling
data.undo (inference.py:70-111), cgcnn.predict_tta builds the same copies
batch by batch in HBM and undoes + averages them there (same batches, same
arithmetic order; see tests/test_gpu_data.py).
"""
import os
import pickle
import pprint
import sys

import numpy as np

from network import models_att
from tools import cli_flags, data, params_help

PACKAGE_DIR = os.path.dirname(os.path.realpath(__file__))


def load_splits(args, reader):
    """Train items (their statistics normalise the inputs) and test items.
    With --subset the reference draws BOTH subsets from the train items
    (inference.py:62-63); the drop-in keeps that so the same command predicts
    the same poses."""
    train = reader.real_read(args.train_set, "train")
    test = reader.real_read(args.test_set, "test")
    if args.subset is not None:
        train = data.get_subset(train, subset_size=args.subset, mode="camera")
        test = data.get_subset(train, subset_size=args.subset, mode="camera")
    return train, test


def draw_translation(args):
    """One uniform shift in [-factor, factor] for the translated copy (inference.py:86-90)."""
    if not args.translate_data:
        return None
    if args.translation_factor < 0:
        raise ValueError("Translation factor must be non-negative")
    return np.random.uniform(-args.translation_factor, args.translation_factor)


def main(argv=None):
    args = cli_flags.parse("inference", argv)
    reader = data.DataReader()
    _, x_test = reader.read_2d(*load_splits(args, reader))
    y_train, _ = reader.read_3d()
    translation = draw_translation(args)

    params = params_help.get_params(is_training=True, gt_dataset=y_train)
    params_help.update_parameters(args, params)
    print(pprint.pformat(params))

    network = models_att.cgcnn(**params)
    print("Start with predictions")
    if args.flip_data or args.rotation_data or args.translate_data:
        predictions = network.predict_tta(x_test, flip=args.flip_data, rotate=args.rotation_data,
                                          translation=translation)
    else:
        predictions = network.predict(data=x_test, sess=None)
    print("Predictions done")

    result = reader.denormalize(predictions)
    if int(os.environ.get("RANK", "0")) == 0:  # one process per GPU: every rank predicted the same
        with open(os.path.join(PACKAGE_DIR, "experiment", params["dir_name"], "result.pkl"), "wb") as f:
            pickle.dump(result, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
