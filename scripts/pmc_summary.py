"""Average PMC counters per kernel over the rocprofv3 passes in a directory."""
import collections, csv, glob, sys

d = sys.argv[1]
agg = collections.defaultdict(float)
n = collections.Counter()
for f in glob.glob(f"{d}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"][:50], r["Counter_Name"])
        agg[k] += float(r["Counter_Value"])
        n[k] += 1
for k in sorted(agg):
    print(f"{k[0]:50s} {k[1]:30s} {agg[k] / n[k]:.4g}")
