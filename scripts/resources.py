"""Register / LDS / occupancy report of every kernel of a HIP source file
(hipcc -Rpass-analysis=kernel-resource-usage), one line per kernel.
usage: python scripts/resources.py lcn-pose_amd/csrc/gemm_bs.hip [...]"""
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lcn-pose_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Xclang", "-target-feature", "-Xclang",
         "-packed-fp32-ops", "-I/opt/rocm/include", "-I" + os.path.join(CSRC, "..", "..", "include"),
         "-I" + CSRC]


def report(path, extra=()):
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-c", path, "-o", "/dev/null",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    cur = None
    rows = []
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
        if not m:
            continue
        k, _, v = m.group(1).partition(":")
        k, v = k.strip(), v.strip()
        if k == "Function Name":
            cur = {"name": subprocess.run(["c++filt", v], capture_output=True,
                                          text=True).stdout.strip().split("(")[0]}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for c in rows:
        print(f"{c['name'][:64]:64s} vgpr {c.get('VGPRs'):>4} agpr {c.get('AGPRs'):>3} sgpr {c.get('TotalSGPRs'):>3} "
              f"spill {c.get('VGPRs Spill'):>3} scratch {c.get('ScratchSize [bytes/lane]'):>4} "
              f"occ {c.get('Occupancy [waves/SIMD]'):>2} lds {c.get('LDS Size [bytes/block]')}")


if __name__ == "__main__":
    extra = [a for a in sys.argv[1:] if a.startswith("-")]
    for p in [a for a in sys.argv[1:] if not a.startswith("-")]:
        report(p, extra)
