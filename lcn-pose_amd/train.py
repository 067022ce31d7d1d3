"""Training CLI of the MI355X-native LCN; takes the flags of the reference's
train.py (train.py:16-40; schema in tools/cli_flags.py).

    python train.py --train_set h36m --validation_set h36m [--knn 3 --layers 3 ...]

Reads <package>/dataset/<set>_{train,val}.pkl (or $LCN_DATASET_DIR), builds the
model parameters as the reference does (params_help.get_params +
update_parameters) and runs network.models_att.cgcnn(**params).fit(...) on
liblcn.so.  Under a launcher that sets WORLD_SIZE > 1 (one process per GPU)
fit steps the global batch data-parallel.
"""
import pprint
import sys

import numpy as np

from network import models_att
from tools import cli_flags, data, params_help

# pre-augmented pickles the reference appends to the train split (train.py:57-63)
EXTRA_SPLITS = (("rotation_data", "train_rotated"), ("translate_data", "train_translation"))


def load_splits(args, reader):
    """Ground-truth item lists of the train and validation splits."""
    train = reader.real_read(args.train_set, "train")
    val = reader.real_read(args.validation_set, "val")
    for flag, split in EXTRA_SPLITS:
        if getattr(args, flag):
            train.extend(reader.real_read(args.train_set, split))
    if args.subset is not None:
        train = data.get_subset(train, subset_size=args.subset, mode="camera")
        val = data.get_subset(val, subset_size=args.subset, mode="camera")
    return train, val


def arrays(args, reader, train, val):
    """Normalised 2-D inputs and 3-D labels; --flip-data appends the mirrored
    copy of the train arrays (train.py:85-87)."""
    x_train, x_val = reader.read_2d(train, val)
    y_train, y_val = reader.read_3d()
    if args.flip_data:
        x_train = np.concatenate((x_train, data.flip_data(x_train.copy())), axis=0)
        y_train = np.concatenate((y_train, data.flip_data(y_train.copy())), axis=0)
    return x_train, y_train, x_val, y_val


def main(argv=None):
    args = cli_flags.parse("train", argv)
    reader = data.DataReader()
    x_train, y_train, x_val, y_val = arrays(args, reader, *load_splits(args, reader))

    params = params_help.get_params(is_training=True, gt_dataset=y_train)
    params_help.update_parameters(args, params)
    print(pprint.pformat(params))

    network = models_att.cgcnn(**params)
    try:
        losses, t_step = network.fit(x_train, y_train, x_val, y_val, args.output_file,
                                     starting_checkpoint=args.resume_from)
    except KeyboardInterrupt:
        print("Training interrupted")
        return 130
    except Exception as e:  # noqa: BLE001 -- the reference reports and stops (train.py:119-121)
        print("Error during training: ", e)
        return 1
    print(losses)
    print(t_step)
    return 0


if __name__ == "__main__":
    sys.exit(main())
