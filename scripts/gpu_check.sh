#!/bin/bash
# On the GPU box: parity tests, bench, rocprof kernel summary. Stops at the first failure.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/check
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
  python3 - <<'PY'
import csv, os
O = os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/check/prof/run_kernel_stats.csv"
rows = list(csv.DictReader(open(O)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:22]:
    print(f"{r['Name'][:58]:58s} n={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:8.1f}us tot={float(r['TotalDurationNs'])/1e6:7.2f}ms {100*float(r['TotalDurationNs'])/tot:5.1f}%")
PY
fi
