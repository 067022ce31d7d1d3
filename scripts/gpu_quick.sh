#!/bin/bash
# On the GPU box: parity tests + one bench line (no CPU leg); ARGS = extra bench arguments.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/quick
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_data.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 $ARGS > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json, os
d = json.load(open(os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/quick/bench.json"))
print("ms_per_step", d["ms_per_step"], "value", d["value"])
print("kernels", {k: v["avg_ms"] for k, v in d["kernels"].items()})
print("thin", [(t["kernel"][:10], t["avg_ms"], t["frac"]) for t in d["hbm_thin_layers"]])
print("bn_act", d["hbm_elementwise"]["avg_ms"], "fwd_only", d.get("fwd_only_poses_per_s"))
PY
