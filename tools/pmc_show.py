"""Print median per-launch counter values of the non-stats trace kernel from gpurun_out/pmc_<cfg>_*."""
import csv
import glob
import statistics
import sys
from collections import defaultdict



def is_frame_kernel(name: str) -> bool:
    """k_trace_frame*<MODE, STATS=false, ...>: the timed frame kernel, not the counter pass."""
    if "k_trace_frame" not in name or "<" not in name:
        return False
    args = [a.strip() for a in name.split("<", 1)[1].split(">", 1)[0].split(",")]
    return len(args) > 1 and args[1] == "false"


cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
vals = defaultdict(list)
for p in sorted(glob.glob(f"gpurun_out/pmc_{cfg}_*/run_counter_collection.csv")):
    for row in csv.DictReader(open(p)):
        k = row["Kernel_Name"]
        if is_frame_kernel(k):
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in vals.items():
    print(f"{k:32s} {statistics.median(v):16.1f}  (n={len(v)})")
