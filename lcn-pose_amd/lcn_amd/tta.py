"""Test-time augmentation descriptors for the device-resident predict path.

inference.py (reference, :70-110) concatenates augmented copies of the test
set -- flip (tools/data.py:10-25), rotation by 180 degrees about joint 0
(:289-322), translation by a random scalar (:27-54) -- in the order the flags
are given, records each copy's position in ``op_ord``, predicts the whole
concatenation and calls ``data.undo`` (:269-287) to map every copy back and
average.  ``augment_ops`` turns the same flags into the per-copy operations
that liblcn applies on the device (lcn_predict_dataset), so the test set is
uploaded once and never concatenated on the host.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from .native import AUG_FLIP, AUG_NONE, AUG_ROTATE, AUG_TRANSLATE

Op = Tuple[int, float, float]


def _rot(angle: float) -> Op:
    th = np.radians(angle)  # numpy's own cos / sin, as data.rotate_data computes them
    return (AUG_ROTATE, float(np.cos(th)), float(np.sin(th)))


def augment_ops(flip: bool = False, rotate: bool = False, translation: Optional[float] = None,
                angle: float = 180.0, undo_angle: float = 180.0
                ) -> Tuple[List[Op], List[Op], Dict[str, int]]:
    """(augment, undo, op_ord) for inference.py's --flip-data / --rotation-data
    / --translate_data (translation = the drawn scalar).  Copy 0 is the data
    itself; the others follow in inference.py's order f, r, t."""
    aug: List[Op] = [(AUG_NONE, 0.0, 0.0)]
    undo: List[Op] = [(AUG_NONE, 0.0, 0.0)]
    op_ord: Dict[str, int] = {}
    if flip:
        aug.append((AUG_FLIP, 0.0, 0.0))
        undo.append((AUG_FLIP, 0.0, 0.0))
        op_ord["f"] = len(aug) - 1
    if rotate:
        aug.append(_rot(angle))
        undo.append(_rot(undo_angle))  # data.undo rotates the copy by `angle` (default 180) again
        op_ord["r"] = len(aug) - 1
    if translation is not None:
        aug.append((AUG_TRANSLATE, float(translation), 0.0))
        undo.append((AUG_TRANSLATE, float(translation), 0.0))  # untranslation_data: - t on x, y, z
        op_ord["t"] = len(aug) - 1
    return aug, undo, op_ord
