"""One training step's kernel timeline from a rocprofv3 kernel trace
(`--kernel-trace --output-format csv`): every kernel between two Adam
launches with its duration and the gap before it, then busy / gap / span.

    python scripts/step_timeline.py gpurun_out/check/prof/run_kernel_trace.csv [step]
"""
import csv
import sys


def main(path, step=5):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    if len(adam) < step + 2:
        raise SystemExit(f"only {len(adam)} Adam launches in {path}")
    i0, i1 = adam[step] + 1, adam[step + 1] + 1
    busy = gaps = 0
    prev = int(rows[i0]["Start_Timestamp"])
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        gaps += max(s - prev, 0)
        print(f"{r['Kernel_Name'][:64]:64s} {(e - s) / 1e3:8.1f} us  gap {(s - prev) / 1e3:6.1f}")
        prev = e
    span = int(rows[i1 - 1]["End_Timestamp"]) - int(rows[i0]["Start_Timestamp"])
    print(f"busy {busy / 1e6:.3f} ms  gaps {gaps / 1e6:.3f} ms  span {span / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
