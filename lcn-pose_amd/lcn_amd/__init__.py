"""lcn_amd -- MI355X-native LCN hot path (HIP kernels behind a C ABI).

``lcn_amd.native.Network`` wraps one liblcn handle (one GPU);
``network.models_att.cgcnn`` (sibling package) is the reference-compatible
model class built on it.
"""
from .native import LcnNativeError, Network, load_library  # noqa: F401

__all__ = ["Network", "LcnNativeError", "load_library"]
