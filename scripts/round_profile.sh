#!/bin/bash
# On the GPU box: the measured evidence in one go -- GPU tests, bench line,
# rocprofv3 kernel stats + trace of the same bench command, PMC traffic.
# Results under gpurun_out/round/ (copy what is to be kept into profiles/).
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/round
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
cd $R
python3 scripts/prof_summary.py $O/prof/run_kernel_trace.csv > $O/kernel_summary.json && cat $O/kernel_summary.json
python3 scripts/step_timeline.py $O/prof/run_kernel_trace.csv > $O/step_timeline.txt 2>/dev/null || true
bash scripts/traffic.sh > $O/traffic.log 2>&1 || { echo "traffic failed"; tail -5 $O/traffic.log; exit 1; }
cp $R/gpurun_out/traffic/traffic.json $O/traffic.json && cat $O/traffic.json
