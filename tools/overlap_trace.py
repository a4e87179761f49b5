#!/usr/bin/env python3
"""Frames in flight, from a rocprofv3 kernel trace: do consecutive frames' trace kernels run
at the same time?

Reads <dir>/run_kernel_trace.csv of a `rocprofv3 --kernel-trace` run over `bench.py --in-flight S`, keeps the
trace-kernel dispatches of the timed region (the last --steps launches of the headline kernel), sorts them by
start and reports, per consecutive pair (k, k + 1): whether frame k + 1's kernel started before frame k's ended,
the overlapped time, and over the whole region: the mean kernel duration, the mean start-to-start period (the
throughput interval), the busy union of all kernels vs the sum of their durations (overlap fraction), and how
many streams (Stream_Id) carried them.

  python3 tools/overlap_trace.py gpurun_out/prof_r03_C2_if3 --steps 200 --out profiles/r03_C2_inflight3_overlap.json
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics


def load(d: str, pattern: str):
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not path:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = []
    with open(path[0]) as f:
        for r in csv.DictReader(f):
            if pattern in r["Kernel_Name"] and "true" not in r["Kernel_Name"].split("<", 1)[-1].split(",")[1]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r.get("Stream_Id", 0) or 0),
                             int(r.get("Queue_Id", 0) or 0), r["Kernel_Name"]))
    return path[0], rows


def summarize(rows, steps: int):
    rows = sorted(rows)[-steps:] if steps else sorted(rows)
    dur = [e - s for s, e, *_ in rows]
    pairs = []
    for (s0, e0, *_), (s1, e1, *_) in zip(rows, rows[1:]):
        pairs.append({"starts_before_prev_ends": s1 < e0, "overlap_ns": max(0, min(e0, e1) - s1)})
    # busy union of all intervals
    union, cur_s, cur_e = 0, None, None
    for s, e, *_ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        union += cur_e - cur_s
    span = rows[-1][1] - rows[0][0]
    period = span / len(rows)
    overlapped = sum(p["starts_before_prev_ends"] for p in pairs)
    return {
        "launches": len(rows),
        "kernel": (re.search(r"(k_\w+<[^>]*>)", rows[0][4]) or re.search(r"(k_\w+)", rows[0][4])).group(1) if rows else None,
        "streams": sorted({r[2] for r in rows}),
        "queues": sorted({r[3] for r in rows}),
        "mean_kernel_ms": round(statistics.mean(dur) / 1e6, 5),
        "median_kernel_ms": round(statistics.median(dur) / 1e6, 5),
        "period_ms": round(period / 1e6, 5),
        "pairs_overlapping": overlapped,
        "pairs": len(pairs),
        "pair_overlap_frac": round(overlapped / max(1, len(pairs)), 4),
        "mean_pair_overlap_ms": round(statistics.mean(p["overlap_ns"] for p in pairs) / 1e6, 5) if pairs else 0.0,
        "sum_kernel_ms": round(sum(dur) / 1e6, 4),
        "busy_union_ms": round(union / 1e6, 4),
        # 1 - union / sum: the share of summed kernel time that ran beside another frame's kernel
        "overlap_frac": round(1.0 - union / max(1, sum(dur)), 4),
        "span_ms": round(span / 1e6, 4),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_trace_frame_packet")
    ap.add_argument("--steps", type=int, default=200, help="launches of the timed region (the last ones)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    path, rows = load(a.dir, a.kernel)
    out = {"source": os.path.relpath(path), **summarize(rows, a.steps)}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
