"""One process per GPU: rank discovery and the RCCL bootstrap.

The reference trains in one process with one TF Session (models_att.py:155,
210-212); here N processes, one per MI355X, each hold a liblcn handle and
step the same global batch together (SyncBN + one gradient all-reduce, see
include/lcn.h).  The launcher (torch.distributed.run, or bench.py's own
spawner) provides RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*; rank 0 creates the
RCCL unique id and publishes it in a file on the node.

Environment overrides (rehearsing several ranks where RCCL cannot join them,
e.g. all on one GPU):
  LCN_COMM=gloo   exchange through torch.distributed's gloo backend on host
                  memory (lcn_comm_init_host) instead of RCCL;
  LCN_DEVICE=d    every rank uses GPU d instead of GPU LOCAL_RANK.
"""
from __future__ import annotations

import os
import sys
import threading
import time

from lcn_amd import native


def bootstrap_timeout():
    """Seconds a rank may spend joining the communicator (LCN_BOOTSTRAP_TIMEOUT,
    default 120): waiting for rank 0's id file and inside ncclCommInitRank, which
    has no bound of its own."""
    return float(os.environ.get("LCN_BOOTSTRAP_TIMEOUT", "120"))


def dist_env():
    """(rank, world, local rank) from the launcher's environment."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LCN_DEVICE", os.environ.get("LOCAL_RANK", str(rank))))
    return rank, world, local


def shard_rows(total, world, rank):
    """Rows of rank `rank` when `total` rows are split over `world` ranks in
    contiguous, near-equal shards (the first total % world ranks hold one more)."""
    base, extra = divmod(total, world)
    return base + (1 if rank < extra else 0)


def shard_slice(total, world, rank):
    """The contiguous slice of rank `rank`'s shard of `total` rows."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return slice(lo, lo + base + (1 if rank < extra else 0))


def uid_path():
    key = "_".join([os.environ.get("MASTER_ADDR", "127.0.0.1"), os.environ.get("MASTER_PORT", "0"),
                    os.environ.get("TORCHELASTIC_RUN_ID", "x"), str(os.getppid())])
    return os.path.join("/tmp", f"lcn_rccl_uid_{key}.bin")


def exchange_uid(rank, world):
    """rank 0 publishes the RCCL unique id in a file every rank on the node can read."""
    path = uid_path()
    if rank == 0:
        uid = native.Network.comm_unique_id()
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    t0, limit = time.time(), bootstrap_timeout()
    while not os.path.exists(path):
        if time.time() - t0 > limit:
            raise RuntimeError(f"rank {rank}: no RCCL unique id from rank 0 within {limit:.0f} s ({path})")
        time.sleep(0.05)
    time.sleep(0.05)
    with open(path, "rb") as f:
        return f.read()


def gloo_allreduce(rank, world):
    """An in-place all-reduce of host numpy arrays over torch.distributed's
    gloo backend (CPU tensors sharing the arrays' memory), for
    Network.comm_init_host.  Joins (or creates) the default process group
    from MASTER_ADDR / MASTER_PORT."""
    import torch
    import torch.distributed as td
    if not td.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        td.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce(arr, op):
        td.all_reduce(torch.from_numpy(arr), op=td.ReduceOp.MAX if op == "max" else td.ReduceOp.SUM)
    return allreduce


class BootstrapWatchdog:
    """Ends this process (exit code 86, a line on stderr) if the block it guards
    has not finished within `seconds`: ncclCommInitRank and the first
    collective wait for every rank without a bound, so one rank that never
    arrives would otherwise hang all the others until the launcher's own limit.
    The launcher (bench.py's spawner, torch.distributed.run) sees the failed
    rank and stops the rest."""

    def __init__(self, rank, seconds, what="communicator setup"):
        self.rank, self.seconds, self.what = rank, seconds, what
        self.timer = None

    def _abort(self):
        sys.stderr.write(f"lcn: rank {self.rank} did not complete the {self.what} within "
                         f"{self.seconds:.0f} s (LCN_BOOTSTRAP_TIMEOUT); exiting\n")
        sys.stderr.flush()
        os._exit(86)

    def __enter__(self):
        if self.seconds > 0:
            self.timer = threading.Timer(self.seconds, self._abort)
            self.timer.daemon = True
            self.timer.start()
        return self

    def __exit__(self, *exc):
        if self.timer is not None:
            self.timer.cancel()
        return False


def mark_ready(rank):
    """Tell a parent that started the ranks (bench.py's spawner sets
    LCN_READY_DIR) that this rank holds its communicator."""
    d = os.environ.get("LCN_READY_DIR")
    if d:
        with open(os.path.join(d, f"ready{rank}"), "w") as f:
            f.write("ok\n")


def comm_setup(net, rank, world):
    """RCCL communicator over the node's ranks; once every rank holds it (the
    host all-reduce below is its first collective) rank 0 removes the id
    file, so a later launch can never read a stale id.  LCN_COMM=gloo: the
    host-exchange communicator over gloo instead.  The whole setup is bounded
    by bootstrap_timeout() (BootstrapWatchdog)."""
    with BootstrapWatchdog(rank, bootstrap_timeout()):
        if os.environ.get("LCN_COMM", "rccl") == "gloo":
            net.comm_init_host(rank, world, gloo_allreduce(rank, world))
            net.allreduce_host([0.0])
        else:
            net.comm_init(exchange_uid(rank, world), rank, world)
            net.allreduce_host([0.0])
            if rank == 0:
                try:
                    os.remove(uid_path())
                except OSError:
                    pass
    mark_ready(rank)
