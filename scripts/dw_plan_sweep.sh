#!/bin/bash
# On the GPU box: weight-gradient plans (lcn_internal.h DwPlan) in gemm_bench.
# CONFIGS="item_rows:rounds ..." ("auto" = the planner's choice; "chunks" = contiguous
# chunks, LCN_DW_SLOTS=0); prints the second round of every case.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R/lcn-pose_amd/csrc
for c in ${CONFIGS:-auto}; do
  E=""
  if [ "$c" = chunks ]; then E="LCN_DW_SLOTS=0"
  elif [ "$c" != auto ]; then IFS=: read item rounds <<< "$c"; E="LCN_DW_ITEM=$item LCN_DW_ROUNDS=$rounds"; fi
  env $E timeout -k 10 120 ./${BUILD:-build}/gemm_bench ${B:-65536} ${ITERS:-20} ${KNN:-3} 1 "${FILTER-dw}" 2 | grep -E "round 1|dw plan|dw mode" | sed "s/^/[$c] /" || exit 1
done
