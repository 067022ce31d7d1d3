"""The C ABI of liblcn.so: every entry point include/lcn.h declares is
exported and bound, and the ctypes structs match the C layout.  CPU only --
nothing here launches a kernel (lcn_create needs a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from lcn_amd import native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "lcn.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\**\s*(lcn_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_abi():
    fns = declared_functions()
    assert "lcn_create" in fns and "lcn_train_step" in fns and "lcn_predict_dataset" in fns
    assert len(fns) >= 28


def test_library_exports_and_binds_every_declared_symbol():
    lib = native.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), f"{name} not exported by liblcn.so"
        assert name in native.SIGNATURES, f"{name} has no ctypes signature"
    assert set(native.SIGNATURES) == set(declared_functions())
    assert lib.lcn_abi_version() == native.LCN_ABI_VERSION


def test_error_paths_need_no_gpu():
    lib = native.load_library()
    h = ctypes.c_void_p()
    assert lib.lcn_create(None, 0, ctypes.byref(h)) == -1          # LCN_E_ARG
    assert b"null" in lib.lcn_last_error(None)
    assert lib.lcn_destroy(None) == 0
    assert lib.lcn_num_params(None) == -1


STRUCT_PROBE = r"""
#include <stddef.h>
#include <stdio.h>
#include "lcn.h"
int main(void) {
  printf("%zu %zu %zu %zu\n", sizeof(lcn_config), offsetof(lcn_config, decay_steps),
         offsetof(lcn_config, mask_matrix), sizeof(lcn_augment));
  printf("%zu %zu\n", offsetof(lcn_augment, param0), offsetof(lcn_augment, param1));
  return 0;
}
"""


def test_ctypes_structs_match_the_c_layout(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(STRUCT_PROBE)
    exe = tmp_path / "probe"
    try:
        subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)],
                       check=True, capture_output=True)
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"no C compiler: {e}")
    a, b = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines()
    size, ds_off, mm_off, aug_size = map(int, a.split())
    p0, p1 = map(int, b.split())
    assert size == ctypes.sizeof(native.LcnConfig)
    assert ds_off == native.LcnConfig.decay_steps.offset
    assert mm_off == native.LcnConfig.mask_matrix.offset
    assert aug_size == ctypes.sizeof(native.LcnAugment)
    assert (p0, p1) == (native.LcnAugment.param0.offset, native.LcnAugment.param1.offset)
