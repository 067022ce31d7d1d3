#!/bin/bash
# On the GPU box: the training step at the per-GPU shard sizes of a strong-
# scaling cfg3 run (65 536 / N rows, N = 8, 4, 2, 1) on one GPU, the reference's
# own small batches, and a kernel trace of the 8 192-row step.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/shards
mkdir -p $O
cd $R
for b in 8192 16384 32768; do
  timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 5 --cpu-baseline 0 > $O/bench_$b.json 2> $O/bench_$b.err || { echo "bench $b failed"; tail -5 $O/bench_$b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$b.json'));print($b, d['ms_per_step'], d['value'], {k:(round(v['avg_ms'],4)) for k,v in d['kernels'].items()})"
done
timeout -k 10 200 python scripts/small_batch.py > $O/small.log 2>&1 || { echo "small failed"; tail -5 $O/small.log; exit 1; }
cat $O/small.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8k -o run --output-format csv -- python3 $R/bench.py --batch 8192 --steps 10 --warmup 2 --cpu-baseline 0 > $O/prof8k.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof8k.log; exit 1; }
python3 - <<'PY'
import csv, os
O = os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/shards/prof8k/run_kernel_stats.csv"
rows = list(csv.DictReader(open(O)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:30]:
    print(f"{r['Name'][:70]:70s} n={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:8.1f}us tot={float(r['TotalDurationNs'])/1e6:7.2f}ms {100*float(r['TotalDurationNs'])/tot:5.1f}%")
PY
