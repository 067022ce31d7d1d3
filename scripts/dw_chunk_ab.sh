#!/bin/bash
# A/B of the thin-layer weight-gradient chunk cap (LCN_DW_MAXCH) under rocprofv3 --stats.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/dwab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in 64 256; do
  LCN_DW_MAXCH=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c$c -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $O/c$c.json 2> $O/c$c.err
  python3 $R/scripts/step_timeline.py $O/c$c/run_kernel_trace.csv 5 > $O/c$c.timeline.txt
  tail -1 $O/c$c.timeline.txt
  grep -E "gemm_dw_kernel<false, (false|true), false>|gemm_bs_kernel<0, 0>|dw_reduce" $O/c$c.timeline.txt | head -20
done
