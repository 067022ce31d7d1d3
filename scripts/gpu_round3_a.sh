#!/bin/bash
# On the GPU box: GPU tests, then the cfg3 / cfg2 bench lines and a one-rank RCCL run.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r3a
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --config cfg2 --steps 20 --warmup 3 --cpu-seconds 9 > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo "cfg2 failed"; tail -20 $O/bench_cfg2.err; exit 1; }
cat $O/bench_cfg2.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --rccl-self 1 > $O/bench_rccl1.json 2> $O/bench_rccl1.err || { echo "rccl-self failed"; tail -20 $O/bench_rccl1.err; exit 1; }
cat $O/bench_rccl1.json
