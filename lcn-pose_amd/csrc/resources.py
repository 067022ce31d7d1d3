"""Per-kernel VGPR/AGPR/scratch/occupancy/LDS summary (compile-time):
python resources.py [files...]"""
import os, re, subprocess, sys

HERE = os.path.dirname(os.path.abspath(__file__))
files = sys.argv[1:] or ["gemm_bs.hip", "kernels_gemm.hip", "kernels_io.hip", "kernels_elem.hip", "kernels_param.hip"]
for f in files:
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "-I../../include", "-c", f, "-o", "/dev/null",
                        "-Rpass-analysis=kernel-resource-usage"], cwd=HERE, capture_output=True, text=True)
    cur, rows = None, []
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        s = m.group(1)
        if s.startswith("Function Name:"):
            cur = {"name": s.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in s:
            k, v = s.split(":", 1)
            cur[k.strip()] = v.strip()
    for d in rows:
        n = re.sub(r"^_ZN3lcn\d+", "", d["name"])[:40]
        g = lambda k: d.get(k, "?")
        print(f"{n:42s} vgpr={g('VGPRs'):>4} agpr={g('AGPRs'):>3} "
              f"scratch={g('ScratchSize [bytes/lane]'):>4} occ={g('Occupancy [waves/SIMD]'):>2} "
              f"lds={g('LDS Size [bytes/block]')}")
