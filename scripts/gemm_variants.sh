#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/gv
mkdir -p $O
make -C $R/lcn-pose_amd/csrc gemm_bench -j16 > $O/build.log 2>&1
timeout -k 10 300 $R/lcn-pose_amd/csrc/build/gemm_bench 65536 10 3 ${NVAR:-7} > $O/variants.txt 2>&1
