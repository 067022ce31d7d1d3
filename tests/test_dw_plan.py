"""The weight-gradient work plan (lcn-pose_amd/csrc/lcn_internal.h: DwPlan,
make_dw_plan, make_dw_wgmap) on the host: every (group, item) covered exactly
once and every partial slot written exactly once, for batch sizes from 1 to
131 072 and group counts of the thin layers, cfg3 and the cfg4 shape.  The
checker is C++ (tests/cpp/dw_plan_check.cpp) compiled host-only with hipcc."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def run_checker(tmp_path, name):
    exe = tmp_path / name
    subprocess.run([HIPCC, "--cuda-host-only", "-O1", "-std=c++17", "-I/opt/rocm/include",
                    "-I" + os.path.join(REPO, "lcn-pose_amd", "csrc"), "-I" + os.path.join(REPO, "include"),
                    "-x", "hip", os.path.join(REPO, "tests", "cpp", name + ".cpp"), "-o", str(exe)],
                   check=True, capture_output=True, text=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not found")
def test_every_item_and_slot_is_covered_once(tmp_path):
    run_checker(tmp_path, "dw_plan_check")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not found")
def test_output_slab_pairs_cover_every_block_once(tmp_path):
    """make_pair_plan (the two-output-slabs-per-workgroup GEMM): every slab in one
    pair, every block in one merged entry, the exact matching's savings."""
    run_checker(tmp_path, "pair_plan_check")
