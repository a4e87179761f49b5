"""Per-launch timeline of LBVH builds from a rocprofv3 kernel trace (tools/build_prof.py under
`rocprofv3 --kernel-trace`): for every build (a run of kernels that starts with k_tri_setup,
k_inst_boxes, k_bounds or k_build_*), each kernel's duration and the idle gap before it, medians over
the builds of the same shape.
  python tools/build_trace.py gpurun_out/<dir>/**/kernel_trace.csv"""
import collections
import csv
import glob
import statistics
import sys

START = ("k_tri_setup", "k_inst_boxes")


def short(name):
    n = name
    for p in ("rt::(anonymous namespace)::", "void "):
        n = n.replace(p, "")
    return n.split("(")[0]


def main(paths):
    rows = []
    for p in paths:
        for q in glob.glob(p, recursive=True):
            with open(q) as f:
                for r in csv.DictReader(f):
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    builds, cur = [], None
    for s, e, n in rows:
        if n.startswith(START) or cur is None:
            if "fillBuffer" in n:
                continue
            cur = []
            builds.append(cur)
        if "k_trace" in n or "k_raster" in n:
            cur = None
            continue
        cur.append((s, e, n))
    shapes = collections.defaultdict(list)
    for b in builds:
        if b:
            shapes[tuple(n for _, _, n in b)].append(b)
    for shape, bs in sorted(shapes.items(), key=lambda kv: -len(kv[1])):
        print(f"== {len(bs)} builds of {len(shape)} launches")
        tot = statistics.median((b[-1][1] - b[0][0]) / 1e3 for b in bs)
        busy = statistics.median(sum(e - s for s, e, _ in b) / 1e3 for b in bs)
        for i, n in enumerate(shape):
            d = statistics.median((b[i][1] - b[i][0]) / 1e3 for b in bs)
            g = statistics.median((b[i][0] - b[i - 1][1]) / 1e3 for b in bs) if i else 0.0
            print(f"  {n:40s} dur {d:8.2f} us  gap {g:6.2f} us")
        print(f"  first start -> last end {tot:.2f} us, kernels busy {busy:.2f} us")


if __name__ == "__main__":
    main(sys.argv[1:] or ["gpurun_out/**/*kernel_trace.csv"])
