"""bench.py's contract on the GPU (the driver parses its last line): one JSON
line with the headline keys, the roofline / HBM / CPU-baseline objects, and
the predict mode; small batch and few steps."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    r = subprocess.run([sys.executable, "bench.py", *args], cwd=REPO, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_train_line_has_the_contract_keys():
    d = _bench("--batch", "4096", "--steps", "3", "--warmup", "1", "--cpu-seconds", "1")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "hbm"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0 and d["dtype"] == "f32"
    assert d["config"]["workload"].startswith("cfg3")
    roof = d["roofline"]
    assert roof["bound"] == "mfma" and roof["unit"] == "TFLOP/s" and 0 < roof["frac"] < 1
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    assert 0 < d["hbm"]["frac"] < 1
    ew = d["hbm_elementwise"]
    assert ew["launches"] == 3 * 4 and 0 < ew["frac"] < 1   # lift + 3 blocks per step


def test_predict_mode():
    d = _bench("--mode", "predict", "--knn", "5", "--batch", "4096", "--steps", "2", "--warmup", "1")
    assert d["value"] > 0 and d["finite"] and d["config"]["copies"] == 3


def test_train_line_with_an_rccl_communicator_is_alone_on_stdout():
    """With a communicator (one rank here; every rank at N > 1) RCCL prints
    its version banner to stdout on rank 0; bench.py must still print only
    the JSON line there."""
    d = _bench("--batch", "4096", "--steps", "2", "--warmup", "1", "--cpu-baseline", "0",
               "--rccl-self", "1")
    assert d["value"] > 0 and "one-rank RCCL" in d["config"]["parallelism"]
    d = _bench("--mode", "predict", "--batch", "2048", "--steps", "1", "--warmup", "1", "--rccl-self", "1")
    assert d["value"] > 0 and d["finite"]
