"""Headline benchmark: poses/s of the 17-joint LCN training step (forward +
backward + Adam) on synthetic data resident in HBM.

Workload (BASELINE.json configs[2], "cfg3"): H36M 17-joint, locally
connected mask, knn=3, layers=3, F=64, batch 65 536 poses per GPU (weak
scaling: the global batch is 65 536 x N with SyncBN over all of it).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU; ranks find each other through RCCL (librccl, bootstrapped
with a unique id passed through a file on the node).  No torch import: the
product path is liblcn.so through ctypes.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lcn-pose_amd"))

from lcn_amd import native  # noqa: E402
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536, help="poses per GPU per step")
    ap.add_argument("--knn", type=int, default=3)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--channels", type=int, default=64)
    ap.add_argument("--mask-type", default="locally_connected")
    ap.add_argument("--rccl-self", type=int, default=0,
                    help="at N=1, create a one-rank RCCL communicator so the step runs the "
                         "multi-GPU path (phased SyncBN, RCCL all-reduces)")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--traffic-file", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--mode", choices=["train", "predict"], default="train",
                    help="train: the headline training step (default); predict: cfg5-style "
                         "inference -- float64 poses resident in HBM, flip + rotation TTA "
                         "(3 copies), batch-statistics BN, undo + average on the device")
    return ap.parse_args()


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def _uid_path():
    key = "_".join([os.environ.get("MASTER_ADDR", "127.0.0.1"), os.environ.get("MASTER_PORT", "0"),
                    os.environ.get("TORCHELASTIC_RUN_ID", "x"), str(os.getppid())])
    return os.path.join("/tmp", f"lcn_rccl_uid_{key}.bin")


def comm_setup(net, rank, world):
    """RCCL communicator over the node's ranks; once every rank holds it (the
    host all-reduce below is its first collective) rank 0 removes the id
    file, so a later launch can never read a stale id."""
    net.comm_init(exchange_uid(rank, world), rank, world)
    net.allreduce_host([0.0])
    if rank == 0:
        try:
            os.remove(_uid_path())
        except OSError:
            pass


def exchange_uid(rank, world):
    """rank 0 publishes the RCCL unique id in a file every rank on the node can read."""
    path = _uid_path()
    if rank == 0:
        uid = native.Network.comm_unique_id()
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > 300:
            raise RuntimeError("timed out waiting for the RCCL unique id")
        time.sleep(0.05)
    time.sleep(0.05)
    with open(path, "rb") as f:
        return f.read()


def cpu_baseline(args, seconds):
    """The numpy restatement (oracle/lcn_oracle.py) timed on this host's cores:
    a bounded sample of the same training step (float32, smaller batch)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import lcn_oracle as O
    cfg = O.Config(F=args.channels, num_layers=args.layers, mask_type=args.mask_type,
                   neighbour=O.neighbour_matrix(args.knn))
    params = O.init_params(cfg, seed=0)
    st = O.adam_init(cfg, params)
    B = 4096
    rng = np.random.default_rng(0)
    x = rng.uniform(-1, 1, (B, 34)).astype(np.float32)
    lab = rng.uniform(-1, 1, (B, 51)).astype(np.float32)
    O.train_step(cfg, params, st, x, lab)  # warm-up
    times = []
    t_end = time.time() + seconds
    while time.time() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        O.train_step(cfg, params, st, x, lab)
        times.append(time.perf_counter() - t0)
        if len(times) >= 20:
            break
    med = float(np.median(times))
    cores = int(os.environ.get("OMP_NUM_THREADS", os.environ.get("OPENBLAS_NUM_THREADS", "0")) or 0) \
        or os.cpu_count()
    return {"value": round(B / med, 1), "unit": "poses/s", "cores": cores, "kind": "port",
            "sample": f"numpy float32 restatement (oracle/lcn_oracle.py), fwd+bwd+Adam, B={B}, "
                      f"{len(times)} steps, median {med:.3f} s/step, OpenBLAS threads={cores}"}


def predict_main(args, rank, world, local):
    """BASELINE.json configs[4] shape (cfg5): TTA predict of `--batch` poses per
    GPU (flip + rotation: 3 copies, inference.py:70-111) through
    lcn_predict_dataset, batch size = --batch, float64 predictions to the host."""
    from lcn_amd.tta import augment_ops
    B = args.batch
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
            "value": round(B * world * args.steps / el, 1), "unit": "poses/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic float64 poses resident in HBM; predictions float64 to the host",
            "config": {"workload": f"cfg5-style inference: locally_connected knn={args.knn}, "
                                   f"layers={args.layers}, F={args.channels}, flip+rotation TTA",
                       "poses_per_gpu": B, "network_batch": B, "copies": 3,
                       "parallelism": f"dp{world} (SyncBN over the ranks' batches)"},
            "finite": bool(np.isfinite(pred).all())})
    net.close()


def main():
    global RESULT_OUT
    args = parse()
    RESULT_OUT = _claim_stdout()
    if args.mode == "predict":
        rank, world, local = dist_env()
        return predict_main(args, rank, world, local)
    rank, world, local = dist_env()
    if world != args.gpus:
        # launched without torchrun: single process drives one GPU
        if world == 1 and args.gpus != 1:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE=1; running 1 GPU", file=sys.stderr)
    B = args.batch
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

    # synthetic poses resident in HBM (x ~ U(-1,1); labels = lifted x + noise)
    rng = np.random.default_rng(1234 + rank)
    x = rng.uniform(-1, 1, (B, 34)).astype(np.float32)
    x3 = x.reshape(B, 17, 2)
    lab = np.concatenate([x3, rng.uniform(-1, 1, (B, 17, 1)).astype(np.float32)], axis=2)
    lab = (lab + 0.1 * rng.standard_normal(lab.shape)).reshape(B, 51).astype(np.float32)
    xb = net.device_buffer(0, x.nbytes)
    lb = net.device_buffer(1, lab.nbytes)
    xb.upload(x)
    lb.upload(lab)

    def barrier():
        net.synchronize()
        net.allreduce_host([0.0])

    for _ in range(args.warmup):
        net.train_step_device(xb.ptr, lb.ptr, B)
    barrier()
    net.set_timing(True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        net.train_step_device(xb.ptr, lb.ptr, B)
    net.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = float(net.allreduce_host([elapsed], op="max")[0])
    kern = {}
    for name, kid in (("gemm_fwd", native.K_GEMM_FWD), ("gemm_dx", native.K_GEMM_DX),
                      ("gemm_dw", native.K_GEMM_DW)):
        n, ms, fl = net.kernel_timing(kid)
        if n:
            kern[name] = {"launches": n, "avg_ms": ms / n, "tflops": fl / (ms * 1e-3) / 1e12,
                          "total_ms_per_step": ms / args.steps}
    bn_act_timing = net.kernel_timing(native.K_BN_ACT)
    net.set_timing(False)

    # forward-only rate (BASELINE configs[1], cfg2) on the same resident batch
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
    value = B * world * args.steps / elapsed
    if rank == 0:
        dom = max(kern, key=lambda k: kern[k]["total_ms_per_step"])
        d = kern[dom]
        traffic = None
        if os.path.exists(args.traffic_file):
            try:
                traffic = json.load(open(args.traffic_file)).get(dom, {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        roof = {"bound": "mfma", "kernel": f"{dom} (block-sparse fp32 v_mfma_f32_32x32x2_f32)",
                "achieved": round(d["tflops"], 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(d["tflops"] / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
                "avg_launch_ms": round(d["avg_ms"], 4)}
        # the metric's "achieved HBM GB/s vs peak", for the hidden-layer forward
        # GEMM (the north star's fused LCN forward): algorithmic bytes = read the
        # input activations + write z, 2 x 17*F floats per pose
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
        hbm = None
        if "gemm_fwd" in kern:
            f = kern["gemm_fwd"]
            alg = 2 * 17 * args.channels * 4 * B
            tr = None
            if os.path.exists(args.traffic_file):
                try:
                    tr = json.load(open(args.traffic_file)).get("gemm_fwd", {}).get("hbm_bytes_per_launch")
                except Exception:
                    tr = None
            ach = alg / (f["avg_ms"] * 1e-3) / 1e9
            hbm = {"kernel": "gemm_fwd (hidden-layer forward: masked GEMM + bias + BN statistics, "
                             "BN apply + LeakyReLU of its input fused)",
                   "algorithmic_bytes": alg, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                   "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": tr,
                   "traffic_GBps": round(tr / (f["avg_ms"] * 1e-3) / 1e9, 1) if tr else None,
                   "mfma_frac": round(f["tflops"] / FP32_PEAK_TFLOPS, 4),
                   "note": "compute-bound: 165 FLOP/B vs a 19.7 FLOP/B fp32 ridge (DESIGN.md)"}
        res = {
            "metric": METRIC, "value": round(value, 1), "unit": "poses/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (x~U(-1,1), labels = lifted x + noise), resident in HBM",
            "config": {"workload": "cfg3: H36M 17-joint LCN train step (fwd+bwd+Adam), "
                                   f"{args.mask_type} knn={args.knn}",
                       "global_batch": B * world, "per_gpu_batch": B, "layers": args.layers,
                       "channels": args.channels, "parallelism": f"dp{world} (SyncBN + RCCL grad all-reduce)"
                       + (", one-rank RCCL communicator" if world == 1 and args.rccl_self else "")},
            "roofline": roof,
            "hbm": hbm,
            "hbm_elementwise": hbm_ew,
            "kernels": {k: {kk: round(vv, 4) if isinstance(vv, float) else vv for kk, vv in v.items()}
                        for k, v in kern.items()},
            "fwd_only_poses_per_s": round(B * world * nf / tfwd, 1),
            "host_input_poses_per_s": round(B * world * nh / thost, 1),
        }
        if args.cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
        else:
            res["cpu_baseline"] = None
        emit(res)
    net.close()


if __name__ == "__main__":
    main()
