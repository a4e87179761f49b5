"""Print median per-launch counter values of the non-stats trace kernel from gpurun_out/pmc_<cfg>_*."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
vals = defaultdict(list)
for p in sorted(glob.glob(f"gpurun_out/pmc_{cfg}_*/run_counter_collection.csv")):
    for row in csv.DictReader(open(p)):
        k = row["Kernel_Name"]
        if "k_trace_frame" in k and "true" not in k:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in vals.items():
    print(f"{k:32s} {statistics.median(v):16.1f}  (n={len(v)})")
