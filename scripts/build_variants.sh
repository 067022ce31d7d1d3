#!/bin/bash
# Build gemm_bench variants HERE (compile-time macros), one build dir each:
#   VARIANTS="base: wo:-DEXP_WAVEORD" bash scripts/build_variants.sh
# then run them on the GPU box with scripts/run_variants.sh.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R/lcn-pose_amd/csrc
for v in ${VARIANTS:-base:}; do
  n=${v%%:*}; f=${v#*:}; f=${f//+/ }
  make gemm_bench BUILD=build_$n EXTRA="$f" -j8 2>&1 | grep -E "error|Error" || true
  test -x build_$n/gemm_bench
done
