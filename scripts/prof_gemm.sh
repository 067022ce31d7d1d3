#!/bin/bash
# On the GPU box: build the GEMM microbench, time it, then collect PMC counters
# in separate rocprofv3 passes (no trace domains mixed with --pmc).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc
mkdir -p $O
make -C $R/lcn-pose_amd/csrc gemm_bench -j16 > $O/build.log 2>&1
BIN=$R/lcn-pose_amd/csrc/build/gemm_bench
timeout -k 10 120 $BIN 65536 20 > $O/gemm_bench.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- $BIN 65536 3 > $O/p$i.log 2>&1 || echo "pass $i failed" >> $O/fail.txt
done
echo done
