#!/bin/bash
# On the GPU box: the step with one / two output slabs per workgroup in the
# hidden layers' forward and backward-data GEMMs, same box, cfg3 and the cfg4 shape.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pair
mkdir -p $O
cd $R
for rep in 1 2; do
  for p in 0 1; do
    LCN_GEMM_PAIR=$p timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 > $O/cfg3_p${p}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('$O/cfg3_p${p}_$rep.json')); print('cfg3 pair=$p', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
  done
done
for p in 0 1; do
  LCN_GEMM_PAIR=$p timeout -k 10 300 python bench.py --config cfg4 --global-batch 16384 --steps 5 --warmup 2 --cpu-baseline 0 > $O/cfg4_p$p.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$O/cfg4_p$p.json')); print('cfg4 pair=$p', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
