#!/bin/bash
# On the GPU box: GEMM microbench timings, then PMC counters per selected case
# (one rocprofv3 pass per counter set; no trace domains mixed with --pmc).
# usage: prof_cases.sh "case substring" ["case substring" ...]
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc
mkdir -p $O
BIN=$R/lcn-pose_amd/csrc/build/gemm_bench
timeout -k 10 120 $BIN 65536 20 3 > $O/gemm_bench.txt 2>&1 || { echo "bench failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
c=0
for cs in "$@"; do
  c=$((c+1))
  i=0
  for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $O/c${c}p$i -o run -- $BIN 65536 5 3 1 "$cs" 1 > $O/c${c}p$i.log 2>&1 || { echo "pass $c/$i failed"; exit 1; }
  done
done
echo done
