#!/bin/bash
# On the GPU box: SQ counters of the forward block-sparse GEMM without epilogue
# (gemm_bench "fwd raw no-epi"), two passes of eight counters, per-kernel means
# and their share of the wave cycles.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() { # name counters...
  n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- $R/lcn-pose_amd/csrc/build/gemm_bench 65536 3 3 1 "fwd raw no-epi" 1 > $O/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/$n.log; return 1; }
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS || exit 1
run b SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE || exit 1
python3 - <<PY
import csv, glob, collections
for n in "ab":
    rows = []
    for f in glob.glob("$O/%s/**/run_counter_collection.csv" % n, recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        agg[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in agg.items():
        m = {x: sum(v) / len(v) for x, v in c.items()}
        wc = m.get("SQ_WAVE_CYCLES", 1)
        print(n, k)
        print("   " + "  ".join(f"{x[3:]}={v:.4g} ({v/wc:.3f})" for x, v in sorted(m.items())))
PY
