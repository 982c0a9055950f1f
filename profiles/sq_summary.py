"""Per-kernel means of the SQ counters captured by profiles/run_sq.sh (gpurun_out/sq_<tag>/g*/...)."""
import collections
import csv
import glob
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
pat = sys.argv[2] if len(sys.argv) > 2 else "k_render_bwd"
vals = collections.defaultdict(list)
for path in glob.glob(f"gpurun_out/sq_{tag}/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if pat in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
