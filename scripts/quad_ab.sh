#!/bin/bash
# On the GPU box: the cfg4 shape with two / four blocks per workgroup in the hidden
# layers' weight gradient (LCN_DW_QUAD=0 / 1), same box; the cfg4-shape GPU tests first.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/quad
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread -k "cfg4 or F128 or F192 or dropout" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for p in 0 1; do
    LCN_DW_QUAD=$p timeout -k 10 300 python bench.py --config cfg4 --batch 16384 --steps 5 --warmup 2 --cpu-baseline 0 > $O/cfg4_q${p}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('$O/cfg4_q${p}_$rep.json')); print('cfg4 quad=$p', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
  done
done
cd lcn-pose_amd/csrc && timeout -k 10 100 ./build/gemm_bench 65536 20 3 1 "dw" 2 | grep "dw4 plan\|round 1"
