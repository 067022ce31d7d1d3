#!/bin/bash
# On the GPU box: run prebuilt gemm_bench variants (scripts/build_variants.sh),
# two rounds each, interleaved.  FILTER selects cases by name.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R/lcn-pose_amd/csrc
for r in 1 2; do
  for v in ${VARIANTS:-base:}; do
    n=${v%%:*}
    timeout -k 10 120 ./build_$n/gemm_bench ${B:-65536} ${ITERS:-20} ${KNN:-3} 1 "${FILTER-dx}" 2 | grep "round 1" | sed "s/^/$n /" || exit 1
  done
done
