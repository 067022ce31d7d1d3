"""The command-line schema of train.py and inference.py as one table.

The two reference CLIs (train.py:16-40, inference.py:16-40) share most of
their flags; a drop-in has to accept the same names with the same types,
choices and defaults.  Each row below is
    (flag, type | "flag", default, extra)
where `default` is either one value for both programs or a dict
{"train": ..., "inference": ...} (a program missing from the dict does not
have the flag), and `extra` holds argparse keywords (choices, required, help).
"""
import argparse

SETS = ["h36m", "humansc3d", "mpii"]
BOTH = ("train", "inference")

FLAGS = [
    ("--test-indices", str, "1", dict(help="experiment/test<idx>/ holds the checkpoints and results")),
    ("--mask-type", str, "locally_connected", dict(choices=["locally_connected", "exponential"])),
    ("--init-type", str, "same", dict(choices={"train": ["same"], "inference": ["same", "ones", "random"]})),
    ("--graph", int, {"inference": 0}, dict(help="index of the skeleton graph")),
    ("--knn", int, 2, dict(help="hops of the joint neighbourhood")),
    ("--layers", int, 3, dict(help="two_linear blocks")),
    ("--in-joints", int, {"inference": 17}, {}),
    ("--out-joints", int, {"inference": 17}, {}),
    ("--dropout", float, {"train": 0, "inference": 0.25}, {}),
    ("--channels", int, 64, dict(help="features per joint")),
    ("--subset", int, None, dict(help="use a subset of this many items per camera")),
    ("--epochs", int, {"train": 25, "inference": 200}, {}),
    ("--checkpoints", str, {"inference": None}, dict(choices=["final", "best"])),
    ("--batch_size", int, 200, {}),
    ("--learning_rate", float, 0.001, {}),
    ("--regularization", float, None, {}),
    ("--in-F", int, 2, dict(choices=[2, 3], help="coordinates per input joint")),
    ("--flip-data", "flag", False, dict(help="left / right flipped copy")),
    ("--rotation-data", "flag", False, dict(help="rotated copy")),
    ("--translate_data", "flag", False, dict(help="translated copy")),
    ("--translation_factor", float, 0.1, {}),
    ("--rotation_factor", float, {"train": 60}, dict(help="degrees")),
    ("--resume_from", str, {"train": None}, dict(help="checkpoint directory to continue from")),
    ("--output_file", str, {"train": None}, dict(help="directory for the loss curves")),
    ("--train_set", str, None, dict(choices=SETS, required=True)),
    ("--validation_set", str, {"train": None}, dict(choices=SETS, required=True)),
    ("--test_set", str, None, dict(choices=SETS, required={"train": False, "inference": True})),
    ("--n_test", int, {"train": 1}, dict(help="runs of a random search")),
]


def _pick(value, program):
    """A per-program dict entry, or the value itself."""
    if isinstance(value, dict) and set(value) <= set(BOTH):
        return value[program]
    return value


def build_parser(program):
    """The argparse parser of `program` ("train" or "inference")."""
    assert program in BOTH
    parser = argparse.ArgumentParser(description=program)
    for flag, kind, default, extra in FLAGS:
        if isinstance(default, dict) and program not in default:
            continue
        kw = {k: _pick(v, program) for k, v in extra.items()}
        if kind == "flag":
            parser.add_argument(flag, action="store_true", default=_pick(default, program), **kw)
        else:
            parser.add_argument(flag, type=kind, default=_pick(default, program), **kw)
    return parser


def parse(program, argv=None):
    return build_parser(program).parse_args(argv)
