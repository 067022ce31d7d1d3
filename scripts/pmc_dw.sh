#!/bin/bash
# On the GPU box: SQ counters of the GEMM microbenchmark's kernels (one pass).
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc_dw
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o run -- $R/lcn-pose_amd/csrc/build/gemm_bench 65536 3 3 1 "${FILTER:-}" 1 > $O/p1.log 2>&1 || { echo "pmc pass failed"; tail -5 $O/p1.log; exit 1; }
python3 - <<PY
import csv, glob, collections
rows = []
for f in glob.glob("$O/p1/**/run_counter_collection.csv", recursive=True) + glob.glob("$O/p1/run_counter_collection.csv"):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1)
    print(k, "n=%d" % len(next(iter(c.values()))))
    print("   " + "  ".join(f"{n[3:]}={v:.3g}" for n, v in sorted(m.items())))
    print("   frac of wave cycles: wait_any %.2f wait_inst %.2f active_inst %.2f wait_inst_lds %.2f | mfma_busy/busy %.2f lds_conflict/wave %.3f" % (
        m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc, m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        m.get("SQ_WAIT_INST_LDS", 0) / wc, m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(m.get("SQ_BUSY_CYCLES", 1), 1),
        m.get("SQ_LDS_BANK_CONFLICT", 0) / wc))
PY
