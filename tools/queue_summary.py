#!/usr/bin/env python3
"""Summarises tools/queue_probe.py's rocprofv3 kernel trace: per kernel name, the durations of the first 20 calls
(the GPU idle) and of the rest (beside trace frames), median and mean in us."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    n = r["Kernel_Name"]
    if "k_trace_frame" in n:
        continue
    by.setdefault(n[:60], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, d in by.items():
    idle, loaded = d[:20], d[20:]
    f = lambda x: (round(statistics.median(x), 1), round(statistics.mean(x), 1)) if x else None  # noqa: E731
    print(f"{n:60s} idle median/mean {f(idle)} us, beside frames {f(loaded)} us ({len(loaded)} calls)")
