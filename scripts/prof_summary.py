"""Per-category kernel durations from a rocprofv3 --kernel-trace CSV, classed
like bench.py's HIP-event timers (scripts/traffic.py classify: hidden-layer
launches = the largest grid of each class), so the rocprof averages can be set
beside bench.py's roofline.avg_launch_ms."""
import csv
import json
import sys

from traffic import classify


def main(trace):
    rows = list(csv.DictReader(open(trace)))
    by = {}
    for r in rows:
        c = classify(r["Kernel_Name"])
        if c is None:
            continue
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        by.setdefault(c, []).append((g, d, r["Kernel_Name"]))
    res = {}
    for c, v in by.items():
        # the thin lift / output launches share kernel (and, for the lift, grid)
        # with the hidden layers but run ~7x shorter: keep the long launches
        gmax = max(g for g, _, _ in v)
        dmax = max(d for g, d, _ in v if g == gmax)
        ds = [d for g, d, _ in v if g == gmax and d > 0.5 * dmax]
        res[c] = {"launches": len(ds), "avg_us": round(sum(ds) / len(ds), 2),
                  "kernels": sorted({n.split("(")[0] for g, d, n in v if g == gmax and d > 0.5 * dmax})}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
