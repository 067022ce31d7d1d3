#!/bin/bash
# On the GPU box: the measured lines besides scripts/round_profile.sh --
# cfg2 / cfg4 / cfg5 lines, the per-GPU shard sizes of a strong-scaling cfg3
# run, the reference's small batches, a one-rank RCCL run.  Results under
# gpurun_out/r3/ (copy what is to be kept into profiles/).
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r3
mkdir -p $O
cd $R
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -20 $O/$name.err; exit 1; }; python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['ms_per_step'], d['value'])"; }
run cfg2 --config cfg2 --steps 20 --warmup 3 --cpu-seconds 12
run cfg4_16384 --config cfg4 --batch 16384 --steps 5 --warmup 2 --cpu-baseline 0
run cfg4_131072 --config cfg4 --steps 3 --warmup 1 --cpu-baseline 0
run cfg5_32768 --config cfg5 --batch 32768 --steps 10 --warmup 2
run cfg5_262144 --config cfg5 --steps 5 --warmup 1
run rccl1 --steps 10 --warmup 3 --cpu-baseline 0 --rccl-self 1
for b in 8192 16384 32768; do run shard_$b --batch $b --steps 30 --warmup 5 --cpu-baseline 0; done
run batch200 --batch 200 --knn 2 --steps 200 --warmup 20 --cpu-baseline 0
run batch512 --batch 512 --knn 1 --steps 200 --warmup 20 --cpu-baseline 0
timeout -k 10 200 python scripts/small_batch.py > $O/small_batch.txt 2>&1 || { echo "small failed"; tail -5 $O/small_batch.txt; exit 1; }
cat $O/small_batch.txt
