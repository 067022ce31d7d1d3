"""Several ranks as PROCESSES on the one GPU of the test box, joined by the
host-exchange communicator over gloo (LCN_COMM=gloo, LCN_DEVICE=0; RCCL
refuses two ranks on one device): bench.py's N > 1 path end to end, and
cgcnn.fit launched as one process per rank against the single-process fit."""
import json
import os
import shutil
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXPERIMENT = os.path.join(REPO, "lcn-pose_amd", "experiment")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR")}
    env.update(LCN_COMM="gloo", LCN_DEVICE="0", **kw)
    return env


def test_bench_gpus_2_runs_two_ranks_and_reports_them():
    """Run plainly, `bench.py --gpus 2` starts its own two ranks: a strong-
    scaling line over the global batch with n_gpus = 2, alone on stdout."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--global-batch", "4096", "--steps", "2",
                        "--warmup", "1", "--cpu-baseline", "0"], cwd=REPO, env=_env(),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    assert d["config"]["global_batch"] == 4096 and d["config"]["per_gpu_batch"] == 2048
    assert d["cpu_baseline"] is None and d["roofline"]["frac"] > 0
    # the exchanges of a step as rank 0 timed them: 4 L + 3 all-reduces, the gradient vector among them
    assert d["comm"] == "host" and d["collectives_per_step"] == 15
    c = d["collectives"]
    assert c["per_step"] == 15 and c["ms_per_step"] > 0 and c["bytes_per_step"] > 4 * 7_000_000


def test_bench_fails_when_a_rank_fails():
    """A rank that cannot start (bad device) ends the whole run non-zero."""
    env = _env()
    env["LCN_DEVICE"] = "63"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--global-batch", "1024", "--steps", "1",
                        "--warmup", "0", "--cpu-baseline", "0"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert not r.stdout.strip()


def _fit(tmp_path, world, tag):
    port = str(_free_port())
    outs, procs = [], []
    name = f"_mp_fit_{tag}_{os.getpid()}"
    for rank in range(world):
        out = tmp_path / f"{tag}_rank{rank}.npz"
        outs.append(out)
        env = _env(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, LCN_INIT_SEED="11", LCN_DROPOUT_SEED="13", FIT_DIR_NAME=name,
                   FIT_JSON_DIR=str(tmp_path / f"json_{tag}"))
        procs.append(subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "mp_fit_worker.py"),
                                       str(out)], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    logs = [p.communicate(timeout=600) for p in procs]
    for p, (so, se) in zip(procs, logs):
        assert p.returncode == 0, se[-3000:]
    res = [np.load(o) for o in outs]
    files = sorted(os.listdir(os.path.join(EXPERIMENT, name, "checkpoints", "final")))
    shutil.rmtree(os.path.join(EXPERIMENT, name), ignore_errors=True)
    return res, logs, files, tmp_path / f"json_{tag}"


def test_fit_as_one_process_per_rank_equals_the_single_process_fit(tmp_path):
    """train.py's cgcnn.fit under WORLD_SIZE = 2 (models_att.py:148-286 made
    data parallel): same batches, each rank steps its shard with SyncBN and
    the gradient all-reduce; only rank 0 prints and writes."""
    (one,), _, files1, _ = _fit(tmp_path, 1, "w1")
    two, logs, files2, jdir = _fit(tmp_path, 2, "w2")
    # rank 0 alone wrote the checkpoint files (one generation: max_to_keep = 1) and the JSON logs
    assert files2 == files1 and len(files2) == 3
    assert sorted(os.listdir(jdir)) == ["training_error.json", "validation_error.json"]
    assert "Total steps" in logs[0][0] and "Total steps" not in logs[1][0]
    for r in two:
        np.testing.assert_array_equal(r["theta"], two[0]["theta"])   # replicas identical
        np.testing.assert_allclose(r["losses"], one["losses"], rtol=2e-5)
        assert np.abs(r["theta"] - one["theta"]).max() <= 2e-5
        assert np.abs(r["pred"] - one["pred"]).max() <= 1e-4
    assert len(one["losses"]) == 2
