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


if __name__ == "__main__":
    sys.exit(pytest.main([__file__, "-q"]))
