#!/bin/bash
# A/B of weight-gradient GEMM loop variants (compile-time macros) with the
# gemm_bench microbenchmark at the cfg3 shape; each variant is its own build:
#   VARIANTS="base: x:-DSOME_MACRO" bash scripts/dw_variants.sh   (one flag per variant)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/dwv
mkdir -p $O
cd $R/lcn-pose_amd/csrc
for v in ${VARIANTS:-base:""}; do
  n=${v%%:*}; f=${v#*:}
  make gemm_bench BUILD=build_$n EXTRA="$f" -j16 > $O/build_$n.log 2>&1
done
for r in 1 2; do
  for v in ${VARIANTS:-base:""}; do
    n=${v%%:*}
    timeout -k 10 120 ./build_$n/gemm_bench 65536 20 3 1 "${FILTER-dw}" 1 | sed "s/^/$n /"
  done
done
