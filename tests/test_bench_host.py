"""bench.py's host-side multi-GPU plumbing on the CPU: the RCCL unique-id
exchange between ranks through a file on the node, and its cleanup once the
communicator exists (no GPU, no RCCL: the id source and the network handle
are stand-ins)."""
import glob
import multiprocessing as mp
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

UID = bytes(range(128))


def _rank(rank, world, q):
    bench.native.Network.comm_unique_id = staticmethod(lambda: UID)
    q.put((rank, bench.exchange_uid(rank, world)))


def test_uid_reaches_every_rank(monkeypatch):
    port = str(40000 + os.getpid() % 20000)
    monkeypatch.setenv("MASTER_PORT", port)
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 3, q)) for r in (2, 1, 0)]  # readers first
    for p in procs:
        p.start()
    got = dict(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: UID, 1: UID, 2: UID}
    # the ranks' parent is this process (as torchrun's agent is theirs)
    for f in glob.glob(f"/tmp/lcn_rccl_uid_*_{port}_*_{os.getpid()}.bin"):
        os.remove(f)


class _FakeNet:
    def __init__(self):
        self.calls = []

    def comm_init(self, uid, rank, world):
        self.calls.append(("init", uid, rank, world))

    def allreduce_host(self, values, op="sum"):
        self.calls.append(("allreduce", list(values)))
        return values


def test_comm_setup_removes_the_id_file(monkeypatch):
    monkeypatch.setenv("MASTER_PORT", str(40001 + os.getpid() % 20000))
    monkeypatch.setattr(bench.native.Network, "comm_unique_id", staticmethod(lambda: UID))
    net = _FakeNet()
    bench.comm_setup(net, 0, 1)
    assert net.calls[0] == ("init", UID, 0, 1)
    assert net.calls[1][0] == "allreduce"     # every rank holds the communicator first
    assert not os.path.exists(bench._uid_path())


def test_claim_stdout_keeps_the_result_line_apart(capfd):
    """Anything written to fd 1 after _claim_stdout goes to stderr; the
    result line goes to the original stdout."""
    saved = os.dup(1)
    try:
        out = bench._claim_stdout()
        os.write(1, b"RCCL version : banner\n")
        out.write('{"value": 1}\n')
        out.flush()
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    captured = capfd.readouterr()
    assert captured.out.strip() == '{"value": 1}'
    assert "RCCL version" in captured.err


RANK_STUB = """
import json, os, sys, time
out = os.environ["STUB_OUT"]
rec = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
rec["argv"] = sys.argv[1:]
with open(os.path.join(out, "rank%s.json" % rec["RANK"]), "w") as f:
    json.dump(rec, f)
if os.environ.get("STUB_HANG_RANK") == rec["RANK"]:
    print("stub rank %s: waiting for a peer that never comes" % rec["RANK"], file=sys.stderr, flush=True)
    time.sleep(60)   # never reports its communicator
if os.environ.get("STUB_HANG_RANK") is not None:
    open(os.path.join(os.environ["LCN_READY_DIR"], "ready" + rec["RANK"]), "w").close()
    time.sleep(60)   # holds its communicator and waits in the first collective
if os.environ.get("STUB_FAIL_RANK") == rec["RANK"]:
    sys.exit(3)
if os.environ.get("STUB_FAIL_RANK") is not None:
    time.sleep(60)   # the surviving ranks would wait in a collective
if rec["RANK"] == "0":
    print(json.dumps({"n_gpus": int(rec["WORLD_SIZE"])}))
"""


def _spawn(tmp_path, monkeypatch, n, fail_rank=None):
    stub = tmp_path / "rank_stub.py"
    stub.write_text(RANK_STUB)
    monkeypatch.setenv("STUB_OUT", str(tmp_path))
    if fail_rank is not None:
        monkeypatch.setenv("STUB_FAIL_RANK", str(fail_rank))
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    argv = ["--gpus", str(n), "--steps", "2"]
    return bench.spawn_ranks(bench.parse(argv), argv, script=str(stub))


def test_gpus_n_starts_n_ranks_with_their_environment(tmp_path, monkeypatch, capfd):
    import json
    assert _spawn(tmp_path, monkeypatch, 4) == 0
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(4)]
    assert [r["RANK"] for r in recs] == ["0", "1", "2", "3"]
    assert [r["LOCAL_RANK"] for r in recs] == ["0", "1", "2", "3"]
    assert {r["WORLD_SIZE"] for r in recs} == {"4"} and {r["MASTER_ADDR"] for r in recs} == {"127.0.0.1"}
    assert len({r["MASTER_PORT"] for r in recs}) == 1
    assert all(r["argv"] == ["--gpus", "4", "--steps", "2"] for r in recs)
    # rank 0's line is the command's stdout
    assert json.loads(capfd.readouterr().out.strip())["n_gpus"] == 4


def test_a_failing_rank_fails_the_run_and_stops_the_others(tmp_path, monkeypatch):
    import time
    t0 = time.time()
    assert _spawn(tmp_path, monkeypatch, 3, fail_rank=1) != 0
    assert time.time() - t0 < 30   # the other ranks were stopped, not waited for


def test_a_rank_that_never_joins_is_stopped_with_its_stderr_tail(tmp_path, monkeypatch, capfd):
    """One rank never reports its communicator: after the bound the spawner stops
    every rank, fails, and shows what each rank last wrote to stderr."""
    import time
    stub = tmp_path / "rank_stub.py"
    stub.write_text(RANK_STUB)
    monkeypatch.setenv("STUB_OUT", str(tmp_path))
    monkeypatch.setenv("STUB_HANG_RANK", "1")
    monkeypatch.setenv("LCN_SPAWN_READY_TIMEOUT", "1.5")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    argv = ["--gpus", "3", "--steps", "2"]
    t0 = time.time()
    assert bench.spawn_ranks(bench.parse(argv), argv, script=str(stub)) != 0
    assert time.time() - t0 < 30
    err = capfd.readouterr().err
    assert "rank(s) [1] had no communicator" in err
    assert "[rank 1] stub rank 1: waiting for a peer that never comes" in err


def test_bootstrap_watchdog_ends_a_rank_stuck_in_the_setup(tmp_path):
    """dist.BootstrapWatchdog: a communicator setup that does not return (as
    ncclCommInitRank does when a peer is missing) ends the process with exit
    code 86 and a line on stderr; a setup that returns in time is left alone."""
    import subprocess
    import time
    code = (
        "import sys, time\n"
        f"sys.path.insert(0, {os.path.join(REPO, 'lcn-pose_amd')!r})\n"
        "from lcn_amd import dist\n"
        "with dist.BootstrapWatchdog(3, float(sys.argv[1])):\n"
        "    time.sleep(float(sys.argv[2]))\n"
        "print('setup done')\n")
    t0 = time.time()
    hung = subprocess.run([sys.executable, "-c", code, "0.5", "60"], capture_output=True, text=True, timeout=60)
    assert hung.returncode == 86 and time.time() - t0 < 30
    assert "rank 3 did not complete the communicator setup" in hung.stderr
    ok = subprocess.run([sys.executable, "-c", code, "30", "0.1"], capture_output=True, text=True, timeout=60)
    assert ok.returncode == 0 and "setup done" in ok.stdout


def test_uid_wait_is_bounded(monkeypatch):
    """A rank whose rank 0 never publishes the id gives up after LCN_BOOTSTRAP_TIMEOUT."""
    monkeypatch.setenv("MASTER_PORT", str(40002 + os.getpid() % 20000))
    monkeypatch.setenv("LCN_BOOTSTRAP_TIMEOUT", "0.3")
    with pytest.raises(RuntimeError, match="no RCCL unique id"):
        bench.exchange_uid(1, 2)


def test_world_size_must_match_gpus(monkeypatch, capsys):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    assert bench.main(["--gpus", "4"]) == 2
    assert "WORLD_SIZE=2" in capsys.readouterr().err


def test_batch_plan_strong_and_weak():
    a = bench.parse([])
    assert a.global_batch == 65536 and a.mode == "train" and (a.knn, a.layers, a.channels) == (3, 3, 64)
    rows = [bench.batch_plan(a, 8, r) for r in range(8)]
    assert rows == [(8192, 65536, "strong")] * 8
    a = bench.parse(["--global-batch", "1000"])
    assert [bench.batch_plan(a, 3, r)[0] for r in range(3)] == [334, 333, 333]
    a = bench.parse(["--batch", "4096"])
    assert bench.batch_plan(a, 4, 2) == (4096, 16384, "weak")
    a = bench.parse(["--config", "cfg2"])
    assert a.mode == "forward" and (a.knn, a.layers, a.channels, a.global_batch) == (3, 3, 64, 65536)
    a = bench.parse(["--config", "cfg4"])
    assert (a.mask_type, a.layers, a.channels, a.global_batch) == ("exponential", 6, 256, 131072)
    a = bench.parse(["--config", "cfg5"])
    assert a.mode == "predict" and a.knn == 5 and a.global_batch == 262144
    with pytest.raises(SystemExit):
        bench.parse(["--batch", "64", "--global-batch", "128"])


if __name__ == "__main__":
    sys.exit(pytest.main([__file__, "-q"]))
