#!/bin/bash
# On the GPU box: fit's step at small batches with and without the small-batch
# GEMM kernel (LCN_SMALL_RT = row-tile limit, 0 = off).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
for rt in 0 1000000; do
  echo "LCN_SMALL_RT=$rt"
  LCN_SMALL_RT=$rt timeout -k 10 200 python scripts/small_batch.py || exit 1
done
