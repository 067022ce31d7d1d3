"""Headline benchmark: poses/s of the 17-joint LCN training step (forward +
backward + Adam) on synthetic data resident in HBM.

Workload (BASELINE.json configs[2], "cfg3"): H36M 17-joint, locally
connected mask, knn=3, layers=3, F=64, GLOBAL batch 65 536 poses per step.
With N GPUs the batch is sharded (rank r takes rows r*G/N ..., SyncBN over
all of it, one RCCL all-reduce of the gradients): strong scaling, the same
model step at every N.  `--batch b` instead keeps b poses per GPU (weak
scaling, global batch b*N -- a different BN batch, hence a different step).
`--config cfg2` is BASELINE.json configs[1] (the forward pass alone, same
batch); `--config cfg4|cfg5` select configs[3] / configs[4].

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU.  Under torch.distributed.run the ranks come from
RANK / LOCAL_RANK / WORLD_SIZE; run plainly with --gpus N > 1, this process
(which never touches the GPU) starts the N ranks itself and fails if any of
them does.  Ranks find each other through RCCL (librccl, bootstrapped with a
unique id passed through a file on the node).  No torch import: the product
path is liblcn.so through ctypes.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lcn-pose_amd"))

from lcn_amd import dist, native  # noqa: E402
from lcn_amd.init import init_flat  # noqa: E402
from tools.params_help import get_neighbour_matrix_by_hand  # noqa: E402
from tools.filter_hub import neighbour_dict_set  # noqa: E402

FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, dense
HBM_PEAK_GBS = 8000.0
HBM_ACHIEVABLE_GBS = 6290.0  # MI355X_MICROARCH.md: float4 copy, measured
METRIC = "poses/sec (17-joint LCN fwd+bwd) at 1/2/4/8 GPU; achieved HBM GB/s vs peak"


def _claim_stdout():
    """Keep stdout for the one JSON line: RCCL prints its version banner to
    stdout from ncclCommInitRank on rank 0, so everything the native side (or
    anything else) writes to fd 1 goes to stderr and the result line is
    written to a private duplicate of the original stdout."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


RESULT_OUT = sys.stdout


def emit(res: dict):
    RESULT_OUT.write(json.dumps(res) + "\n")
    RESULT_OUT.flush()


# BASELINE.json configs[1..4]: model shape, global batch, bench mode
CONFIGS = {
    "cfg2": dict(knn=3, layers=3, channels=64, mask_type="locally_connected", global_batch=65536,
                 mode="forward"),
    "cfg3": dict(knn=3, layers=3, channels=64, mask_type="locally_connected", global_batch=65536,
                 mode="train"),
    "cfg4": dict(knn=2, layers=6, channels=256, mask_type="exponential", global_batch=131072,
                 mode="train"),
    "cfg5": dict(knn=5, layers=3, channels=64, mask_type="locally_connected", global_batch=262144,
                 mode="predict"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="cfg3",
                    help="BASELINE.json config: model shape, global batch and mode defaults")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="poses per step over all GPUs, sharded across them (strong scaling; "
                         "default: the config's)")
    ap.add_argument("--batch", type=int, default=None,
                    help="poses per GPU per step (weak scaling: global batch = batch x GPUs)")
    ap.add_argument("--knn", type=int, default=None)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--channels", type=int, default=None)
    ap.add_argument("--mask-type", default=None)
    ap.add_argument("--rccl-self", type=int, default=0,
                    help="at N=1, create a one-rank RCCL communicator so the step runs the "
                         "multi-GPU path (phased SyncBN, RCCL all-reduces)")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=30.0)
    ap.add_argument("--traffic-file", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--mode", choices=["train", "forward", "predict"], default=None,
                    help="train: the headline training step (default); forward: cfg2, the "
                         "forward pass alone on the resident batch; predict: cfg5-style "
                         "inference -- float64 poses resident in HBM, flip + rotation TTA "
                         "(3 copies), batch-statistics BN, undo + average on the device")
    args = ap.parse_args(argv)
    preset = CONFIGS[args.config]
    for k in ("knn", "layers", "channels", "mask_type", "mode"):
        if getattr(args, k) is None:
            setattr(args, k, preset[k])
    if args.batch is not None and args.global_batch is not None:
        ap.error("--batch (per GPU, weak scaling) and --global-batch (sharded, strong scaling) exclude each other")
    if args.batch is None and args.global_batch is None:
        args.global_batch = preset["global_batch"]
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    return args


dist_env = dist.dist_env
shard_rows = dist.shard_rows


def batch_plan(args, world, rank):
    """(rows of this rank, global rows, scaling label)."""
    if args.batch is not None:
        return args.batch, args.batch * world, "weak"
    if args.global_batch < world:
        raise SystemExit(f"--global-batch {args.global_batch} < {world} ranks")
    return shard_rows(args.global_batch, world, rank), args.global_batch, "strong"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tail(path, n=40):
    try:
        with open(path, errors="replace") as f:
            return f.readlines()[-n:]
    except OSError:
        return []


def spawn_ranks(args, argv, script=None):
    """`bench.py --gpus N` run plainly: start the N ranks as fresh child
    processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment,
    stdout inherited so rank 0's JSON line is this command's), wait for all of
    them, and fail if any fails.  This process makes no GPU call.

    The bootstrap is bounded: a rank that is still running but has not reported
    its communicator (dist.mark_ready) LCN_SPAWN_READY_TIMEOUT seconds after the
    start (default: LCN_BOOTSTRAP_TIMEOUT + 60) counts as hung; the children are
    then terminated and the run fails with every rank's last stderr lines.  The
    ranks' stderr goes through per-rank files that are replayed to this
    process's stderr at the end."""
    import shutil
    import tempfile
    port = str(_free_port())
    ready_limit = float(os.environ.get("LCN_SPAWN_READY_TIMEOUT", dist.bootstrap_timeout() + 60))
    tmp = tempfile.mkdtemp(prefix="lcn_ranks_")
    procs, errs = [], []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   LCN_READY_DIR=tmp)
        errs.append(open(os.path.join(tmp, f"rank{r}.err"), "w"))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__), *argv],
                                      env=env, stderr=errs[-1]))

    def stop_running(codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                p.terminate()
        for i, p in enumerate(procs):
            if codes[i] is None:
                try:
                    codes[i] = p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    codes[i] = p.wait()

    def replay(tails_only):
        for r, f in enumerate(errs):
            f.close()
            path = os.path.join(tmp, f"rank{r}.err")
            lines = _tail(path) if tails_only else _tail(path, 10 ** 9)
            for ln in lines:
                sys.stderr.write(f"[rank {r}] {ln}" if tails_only else ln)
        sys.stderr.flush()
        shutil.rmtree(tmp, ignore_errors=True)

    t0 = time.time()
    codes = [None] * len(procs)
    rc = 0
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        failed = [i for i, c in enumerate(codes) if c not in (None, 0)]
        if failed:  # a rank died: the others would wait in a collective for ever
            stop_running(codes)
            print(f"bench.py: rank(s) {failed} failed with exit code(s) "
                  f"{[codes[i] for i in failed]}", file=sys.stderr)
            rc = 1
            break
        late = [i for i, c in enumerate(codes)
                if c is None and not os.path.exists(os.path.join(tmp, f"ready{i}"))]
        if late and time.time() - t0 > ready_limit:
            stop_running(codes)
            print(f"bench.py: rank(s) {late} had no communicator {ready_limit:.0f} s after the start "
                  f"(LCN_SPAWN_READY_TIMEOUT); all ranks stopped", file=sys.stderr)
            rc = 1
            break
        time.sleep(0.05)
    replay(tails_only=rc != 0)
    return rc


# the RCCL bootstrap lives with the product (cgcnn uses it too)
_uid_path = dist.uid_path
exchange_uid = dist.exchange_uid
comm_setup = dist.comm_setup


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _blas_name():
    try:
        cfg = np.show_config(mode="dicts")
        b = cfg.get("Build Dependencies", {}).get("blas", {})
        return f"{b.get('name', 'unknown')} {b.get('version', '')}".strip()
    except Exception:  # noqa: BLE001
        return "unknown"


def cpu_baseline(args, seconds, batches=(256, 4096, 65536), forward_only=False):
    """The numpy restatement (oracle/lcn_oracle.py) of the same training step
    (float32, forward + backward + Adam; forward_only: the forward pass alone)
    timed on this host's cores: at cfg1's batch 256, at 4 096, and at the
    headline batch 65 536.  `seconds` bounds the whole leg (each size gets a
    third; a size whose first step already exceeds what is left is skipped).
    `value` is the largest batch timed."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import lcn_oracle as O
    cfg = O.Config(F=args.channels, num_layers=args.layers, mask_type=args.mask_type,
                   neighbour=O.neighbour_matrix(args.knn))
    params = O.init_params(cfg, seed=0)
    st = O.adam_init(cfg, params)
    cores = int(os.environ.get("OMP_NUM_THREADS", os.environ.get("OPENBLAS_NUM_THREADS", "0")) or 0) \
        or os.cpu_count()
    rng = np.random.default_rng(0)
    samples = []
    per_size = seconds / len(batches)
    est = None  # seconds per pose of the previous size
    for B in batches:
        if samples and est is not None and est * B * 3 > seconds:
            break  # warm-up + two timed steps of this size would not fit the leg
        x = rng.uniform(-1, 1, (B, 34)).astype(np.float32)
        lab = rng.uniform(-1, 1, (B, 51)).astype(np.float32)

        def one():
            if forward_only:
                O.forward(cfg, params, x, np.float32)
            else:
                O.train_step(cfg, params, st, x, lab)
        one()  # warm-up
        times = []
        t_end = time.time() + per_size
        while (time.time() < t_end or len(times) < 2) and len(times) < 20:
            t0 = time.perf_counter()
            one()
            times.append(time.perf_counter() - t0)
        med = float(np.median(times))
        est = med / B
        samples.append({"batch": B, "steps": len(times), "median_s_per_step": round(med, 4),
                        "poses_per_s": round(B / med, 1)})
    top = samples[-1]
    return {"value": top["poses_per_s"], "unit": "poses/s", "cores": cores, "kind": "port",
            "cpu": _cpu_model(), "blas": _blas_name(), "samples": samples,
            "sample": f"numpy float32 restatement (oracle/lcn_oracle.py), "
                      f"{'forward' if forward_only else 'fwd+bwd+Adam'}, "
                      f"B={top['batch']}, {top['steps']} steps, median {top['median_s_per_step']:.3f} "
                      f"s/step, {_blas_name()} threads={cores}, {_cpu_model()}"}


def predict_main(args, rank, world, local):
    """BASELINE.json configs[4] shape (cfg5): TTA predict of `--batch` poses per
    GPU (flip + rotation: 3 copies, inference.py:70-111) through
    lcn_predict_dataset, batch size = --batch, float64 predictions to the host."""
    from lcn_amd.tta import augment_ops
    B, G, scaling = batch_plan(args, world, rank)
    neighbour = get_neighbour_matrix_by_hand(neighbour_dict_set[0], knn=args.knn)
    mask = (neighbour.T != 0).astype(np.float32)
    net = native.Network(F=args.channels, in_F=2, num_layers=args.layers, mask_type=args.mask_type,
                         mask_matrix=mask, max_batch=B, device=local)
    if world > 1 or args.rccl_self:
        comm_setup(net, rank, world)
    net.set_params(init_flat(net.param_layout(), net.n_params, neighbour, seed=0))
    rng = np.random.default_rng(99 + rank)
    x = rng.uniform(-1, 1, (B, 34))                      # float64, as DataReader yields
    net.dataset_upload(0, x)
    aug, undo, _ = augment_ops(flip=True, rotate=True)
    for _ in range(args.warmup):
        net.predict_dataset(0, B, B, augment=aug, undo=undo)
    net.allreduce_host([0.0])
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pred = net.predict_dataset(0, B, B, augment=aug, undo=undo)
    net.synchronize()
    net.allreduce_host([0.0])
    el = float(net.allreduce_host([time.perf_counter() - t0], op="max")[0])
    if rank == 0:
        emit({
            "metric": "poses/sec, TTA predict (flip + rotation, 3 copies per pose)",
            "value": round(G * args.steps / el, 1), "unit": "poses/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic float64 poses resident in HBM; predictions float64 to the host",
            "config": {"workload": f"cfg5-style inference: locally_connected knn={args.knn}, "
                                   f"layers={args.layers}, F={args.channels}, flip+rotation TTA",
                       "global_poses": G, "poses_per_gpu": B, "network_batch": B, "copies": 3,
                       "parallelism": f"dp{world} (SyncBN over the ranks' batches)"},
            "finite": bool(np.isfinite(pred).all()), **comm_fields(net)})
    net.close()


def make_net(args, rank, world, local, B):
    """The network of the config with its communicator and seeded parameters."""
    neighbour = get_neighbour_matrix_by_hand(neighbour_dict_set[0], knn=args.knn)
    if "locally_connected" in args.mask_type:
        mask = (neighbour.T != 0).astype(np.float32)
    else:
        from network.models_att import get_exponential_matrix
        mask = get_exponential_matrix(verbose=False)
    net = native.Network(F=args.channels, in_F=2, num_layers=args.layers, mask_type=args.mask_type,
                         mask_matrix=mask, max_batch=B, device=local)
    if world > 1 or args.rccl_self:
        comm_setup(net, rank, world)
    net.set_params(init_flat(net.param_layout(), net.n_params, neighbour, seed=0))
    return net


def comm_fields(net):
    """What joined the ranks, as the communicator itself reports it: after an
    RCCL run `rccl_ranks` is ncclCommCount of the live communicator."""
    kind, _, w = net.comm_info()
    return {"comm": kind, "rccl_ranks": w if kind == "rccl" else None}


def synthetic_inputs(net, B, rank):
    """Synthetic poses resident in HBM (x ~ U(-1,1); labels = lifted x + noise)."""
    rng = np.random.default_rng(1234 + rank)
    x = rng.uniform(-1, 1, (B, 34)).astype(np.float32)
    x3 = x.reshape(B, 17, 2)
    lab = np.concatenate([x3, rng.uniform(-1, 1, (B, 17, 1)).astype(np.float32)], axis=2)
    lab = (lab + 0.1 * rng.standard_normal(lab.shape)).reshape(B, 51).astype(np.float32)
    xb = net.device_buffer(0, x.nbytes)
    lb = net.device_buffer(1, lab.nbytes)
    xb.upload(x)
    lb.upload(lab)
    return x, lab, xb, lb


GEMM_IDS = (("gemm_fwd", native.K_GEMM_FWD), ("gemm_dx", native.K_GEMM_DX), ("gemm_dw", native.K_GEMM_DW))
THIN_IDS = (("lift (x . W1e + b1, BN statistics)", native.K_LIFT),
            ("output (h . W4e)", native.K_OUT), ("output weight gradient (h^T dy)", native.K_OUT_DW))


def read_timers(net, steps):
    """The HIP-event timers of the timed region, per kernel class."""
    kern = {}
    for name, kid in GEMM_IDS:
        n, ms, fl = net.kernel_timing(kid)
        if n:
            kern[name] = {"launches": n, "avg_ms": ms / n, "tflops": fl / (ms * 1e-3) / 1e12,
                          "total_ms_per_step": ms / steps}
    bn_act_timing = net.kernel_timing(native.K_BN_ACT)
    thin_timing = {name: net.kernel_timing(kid) for name, kid in THIN_IDS}
    return kern, bn_act_timing, thin_timing


def collective_timing(net, steps):
    """The all-reduces of the timed steps on this rank (HIP events around each
    on the compute stream: enqueue to completion, so with the wait for the
    slowest rank), or None on a handle that is not joined."""
    n, ms, nbytes = net.kernel_timing(native.K_COMM)
    if not n:
        return None
    return {"per_step": n / steps, "ms_per_step": round(ms / steps, 4), "avg_us": round(1e3 * ms / n, 2),
            "bytes_per_step": int(nbytes / steps)}


def pmc_traffic(args, B, kernel):
    """HBM bytes per launch of `kernel` from the committed PMC passes -- they
    were collected on the cfg3 model shape at 65 536 rows and apply only there."""
    applies = (B == 65536 and args.channels == 64 and args.knn == 3 and args.layers == 3
               and args.mask_type == "locally_connected")
    if not applies or not os.path.exists(args.traffic_file):
        return None
    try:
        return json.load(open(args.traffic_file)).get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:  # noqa: BLE001
        return None


def roofline_blocks(args, B, kern, bn_act_timing, thin_timing):
    """`roofline` of the dominant GEMM class and the HBM-side blocks of the line."""
    dom = max(kern, key=lambda k: kern[k]["total_ms_per_step"])
    d = kern[dom]
    roof = {"bound": "mfma", "kernel": f"{dom} (block-sparse fp32 v_mfma_f32_32x32x2_f32)",
            "achieved": round(d["tflops"], 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(d["tflops"] / FP32_PEAK_TFLOPS, 4), "traffic": pmc_traffic(args, B, dom),
            "avg_launch_ms": round(d["avg_ms"], 4)}
    hbm_ew = None
    nba, msba, bytes_ba = bn_act_timing
    if nba:
        gbs = bytes_ba / (msba * 1e-3) / 1e9
        hbm_ew = {"kernel": "bn_act (BN apply + LeakyReLU + residual add, materialising the block "
                            "outputs of the fused forward)", "launches": nba,
                  "avg_ms": round(msba / nba, 4), "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                  "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                  "frac_of_achievable": round(gbs / HBM_ACHIEVABLE_GBS, 4),
                  "achievable": HBM_ACHIEVABLE_GBS}
    # the thin lift / output layers against HBM: algorithmic bytes = input
    # rows read + output rows written.  Their narrow side is padded to the
    # MFMA tile (34 -> 40 input features, 51 -> 64 output columns), which
    # puts a matrix-core floor under each launch: mfma_floor_ms.
    H = 17 * args.channels
    kin = -(-17 * 2 // 8) * 8
    pad_flops = {"lift": 2.0 * kin * H, "output": 2.0 * H * 64}
    hbm_thin = []
    for name, (nt, mst, bt) in thin_timing.items():
        if nt:
            gbs = bt / (mst * 1e-3) / 1e9
            fl = pad_flops["lift" if name.startswith("lift") else "output"] * B
            hbm_thin.append({"kernel": name, "launches": nt, "avg_ms": round(mst / nt, 4),
                             "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(gbs / HBM_PEAK_GBS, 4),
                             "mfma_floor_ms": round(fl / (FP32_PEAK_TFLOPS * 1e12) * 1e3, 4)})
    # the metric's "achieved HBM GB/s vs peak", for the hidden-layer forward
    # GEMM (the north star's fused LCN forward): algorithmic bytes = read the
    # input activations + write z, 2 x 17*F floats per pose
    hbm = None
    if "gemm_fwd" in kern:
        f = kern["gemm_fwd"]
        alg = 2 * 17 * args.channels * 4 * B
        tr = pmc_traffic(args, B, "gemm_fwd")
        ach = alg / (f["avg_ms"] * 1e-3) / 1e9
        hbm = {"kernel": "gemm_fwd (hidden-layer forward: masked GEMM + bias + BN statistics, "
                         "BN apply + LeakyReLU of its input fused)",
               "algorithmic_bytes": alg, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
               "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": tr,
               "traffic_GBps": round(tr / (f["avg_ms"] * 1e-3) / 1e9, 1) if tr else None,
               "mfma_frac": round(f["tflops"] / FP32_PEAK_TFLOPS, 4),
               "note": "compute-bound: 165 FLOP/B vs a 19.7 FLOP/B fp32 ridge (157.3 TFLOP/s over 8 TB/s)"}
    return {"roofline": roof, "hbm": hbm, "hbm_elementwise": hbm_ew, "hbm_thin_layers": hbm_thin,
            "kernels": {k: {kk: round(vv, 4) if isinstance(vv, float) else vv for kk, vv in v.items()}
                        for k, v in kern.items()}}


def forward_main(args, rank, world, local):
    """BASELINE.json configs[1] (cfg2): the forward pass alone -- lift, the
    2L hidden layers with their batch-statistics BN, output layer and output
    assembly (cgcnn.predict's graph, models_att.py:707-775) -- on a batch
    resident in HBM, predictions left on the device."""
    B, G, scaling = batch_plan(args, world, rank)
    net = make_net(args, rank, world, local, B)
    _, _, xb, _ = synthetic_inputs(net, B, rank)
    out = net.device_buffer(2, B * 51 * 4)

    def barrier():
        net.synchronize()
        net.allreduce_host([0.0])

    for _ in range(args.warmup):
        net.forward_device(xb.ptr, out.ptr, B)
    barrier()
    net.set_timing(True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        net.forward_device(xb.ptr, out.ptr, B)
    net.synchronize()
    barrier()
    elapsed = float(net.allreduce_host([time.perf_counter() - t0], op="max")[0])
    kern, bn_act_timing, thin_timing = read_timers(net, args.steps)
    net.set_timing(False)
    if rank == 0:
        res = {
            "metric": METRIC, "value": round(G * args.steps / elapsed, 1), "unit": "poses/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (x~U(-1,1)), resident in HBM; predictions stay on the device",
            "config": {"workload": f"{args.config}: H36M 17-joint LCN forward only, "
                                   f"{args.mask_type} knn={args.knn}",
                       "global_batch": G, "per_gpu_batch": B, "layers": args.layers,
                       "channels": args.channels, "parallelism": f"dp{world} (SyncBN)"},
            **roofline_blocks(args, B, kern, bn_act_timing, thin_timing), **comm_fields(net)}
        res["cpu_baseline"] = (cpu_baseline(args, args.cpu_seconds, forward_only=True)
                               if args.cpu_baseline and world == 1 else None)
        emit(res)
    net.close()


def main(argv=None):
    global RESULT_OUT
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args, argv)
    rank, world, local = dist_env()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
              f"(torch.distributed.run --nproc-per-node {args.gpus}) or run plainly", file=sys.stderr)
        return 2
    RESULT_OUT = _claim_stdout()
    if args.mode == "predict":
        predict_main(args, rank, world, local)
        return 0
    if args.mode == "forward":
        forward_main(args, rank, world, local)
        return 0
    B, G, scaling = batch_plan(args, world, rank)
    net = make_net(args, rank, world, local, B)
    x, lab, xb, lb = synthetic_inputs(net, B, rank)

    def barrier():
        net.synchronize()
        net.allreduce_host([0.0])

    for _ in range(args.warmup):
        net.train_step_device(xb.ptr, lb.ptr, B)
    barrier()
    # Timed region: HIP-event timers on the library's compute stream around
    # every kernel class (timing-only events without a system fence: measured
    # free, 16.45-16.50 ms per step with all classes timed against 16.46-16.52
    # with the roofline's kernel alone)
    net.set_timing(True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        net.train_step_device(xb.ptr, lb.ptr, B)
    net.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = float(net.allreduce_host([elapsed], op="max")[0])
    kern, bn_act_timing, thin_timing = read_timers(net, args.steps)
    comm_timing = collective_timing(net, args.steps)
    net.set_timing(False)

    # forward-only rate (BASELINE configs[1], cfg2: `--config cfg2` gives it a
    # line of its own) on the same resident batch
    out = net.device_buffer(2, B * 51 * 4)
    for _ in range(2):
        net.forward_device(xb.ptr, out.ptr, B)
    barrier()
    tf0 = time.perf_counter()
    nf = max(5, args.steps)
    for _ in range(nf):
        net.forward_device(xb.ptr, out.ptr, B)
    net.synchronize()
    barrier()
    tfwd = float(net.allreduce_host([time.perf_counter() - tf0], op="max")[0])

    # PCIe-inclusive rate: the same step fed from host (pageable) arrays, as
    # cgcnn.fit does per step (H2D copy of x and labels + step + sync)
    for _ in range(1):
        net.train_step(x, lab, want_loss=False)
    barrier()
    th0 = time.perf_counter()
    nh = max(3, args.steps // 2)
    for _ in range(nh):
        net.train_step(x, lab, want_loss=False)
    net.synchronize()
    barrier()
    thost = float(net.allreduce_host([time.perf_counter() - th0], op="max")[0])

    ms_step = elapsed / args.steps * 1e3
    value = G * args.steps / elapsed
    if rank == 0:
        res = {
            "metric": METRIC, "value": round(value, 1), "unit": "poses/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (x~U(-1,1), labels = lifted x + noise), resident in HBM",
            "config": {"workload": f"{args.config}: H36M 17-joint LCN train step (fwd+bwd+Adam), "
                                   f"{args.mask_type} knn={args.knn}",
                       "global_batch": G, "per_gpu_batch": B, "layers": args.layers,
                       "channels": args.channels, "parallelism": f"dp{world} (SyncBN + RCCL grad all-reduce)"
                       + (", one-rank RCCL communicator" if world == 1 and args.rccl_self else "")},
            **roofline_blocks(args, B, kern, bn_act_timing, thin_timing), **comm_fields(net),
            "collectives_per_step": (4 * args.layers + 3) if (world > 1 or args.rccl_self) else 0,
            "collectives": comm_timing,
            "fwd_only_poses_per_s": round(G * nf / tfwd, 1),
            "host_input_poses_per_s": round(G * nh / thost, 1),
        }
        if args.cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
        else:
            res["cpu_baseline"] = None
        emit(res)
    net.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
