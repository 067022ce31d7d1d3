#!/bin/bash
# On the GPU box: HBM traffic of the bench's kernels from PMC counters, one
# rocprofv3 pass per counter (FETCH_SIZE and WRITE_SIZE cannot share a pass),
# summarised by scripts/traffic.py into gpurun_out/traffic/traffic.json.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/traffic
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 > $O/fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 > $O/write.log 2>&1 || { echo "write pass failed"; tail -5 $O/write.log; exit 1; }
python3 $R/scripts/traffic.py $O > $O/traffic.json && cat $O/traffic.json
