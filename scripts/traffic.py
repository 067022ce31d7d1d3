"""HBM bytes per launch of the bench's GEMM kernels from rocprofv3 PMC CSVs.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports
half the bytes of 16-B-per-lane streaming reads, so reads = 2 x FETCH_SIZE;
WRITE_SIZE is exact for 16-B stores.  Both counters are in KiB.  Launch
classes follow bench.py's timer categories: gemm_dw = the hidden-layer
weight-gradient launches (the largest dW grid), gemm_fwd = forward launches
of the hidden layers (gemm_bs_kernel<*, 1> with the largest grid), gemm_dx =
gemm_bs_kernel<0, 2, *> with the largest grid.
"""
import collections
import csv
import glob
import json
import sys


def load(d, counter):
    rows = []
    for f in glob.glob(f"{d}/run_counter_collection.csv") + glob.glob(f"{d}/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["Grid_Size"]),
                             float(r["Counter_Value"]) * 1024.0))
    return rows


def classify(name):
    if "gemm_dw_kernel" in name:
        return "gemm_dw"
    if "gemm_bs_kernel" in name:
        targs = name.split("<")[1].split(">")[0].replace(" ", "").split(",")
        if len(targs) > 1 and targs[1] in ("2", "3"):  # <PRO, EPI, KG>: EPI_BNBACK (3: with dropout)
            return "gemm_dx"
        return "gemm_fwd"
    return None


def main(out_dir):
    fetch = load(f"{out_dir}/fetch", "FETCH_SIZE")
    write = load(f"{out_dir}/write", "WRITE_SIZE")
    res = {}
    for cls in ("gemm_fwd", "gemm_dx", "gemm_dw"):
        per = {}
        for tag, rows, scale in (("read", fetch, 2.0), ("write", write, 1.0)):
            sel = [(g, v) for (_, n, g, v) in rows if classify(n) == cls]
            if not sel:
                continue
            # the thin lift / output launches share kernel and grid with the
            # hidden layers but move a fraction of the bytes: keep the big launches
            gmax = max(g for g, _ in sel)
            vmax = max(v for g, v in sel if g == gmax)
            vals = [v * scale for g, v in sel if g == gmax and v > 0.5 * vmax]
            per[tag] = sum(vals) / len(vals)
            per["launches_" + tag] = len(vals)
        if "read" in per and "write" in per:
            res[cls] = {"read_bytes_per_launch": per["read"], "write_bytes_per_launch": per["write"],
                        "hbm_bytes_per_launch": per["read"] + per["write"],
                        "launches": per["launches_read"]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
