"""Per-frame GPU timeline of the tiled-frame loop under rocprofv3 (tools/native_strips_cost.py --size WxH run under
`rocprofv3 --kernel-trace`): which hardware queue each render / gather / assembly ran on, their durations and the
frame period, over the native 3-stream phase (the last 100 RCCL kernels).
  python3 tools/trace_share.py gpurun_out/prof_share8"""
import csv
import glob
import re
import statistics as S
import sys


def main(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))

    def nm(r):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        return m.group(1) if m else ("rccl" if "rccl" in r["Kernel_Name"] else r["Kernel_Name"][:30])
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], nm(r)) for r in rows)
    rc = [i for i, k in enumerate(ks) if k[3] == "rccl"]
    lo, hi = rc[-100], rc[-1]
    win = ks[lo:hi]
    out = {}
    for kind in ("k_trace_frame_packet", "rccl", "k_assemble16"):
        sel = [k for k in win if k[3] == kind]
        out[kind] = {"n": len(sel), "mean_us": round(S.mean((e - s) / 1000 for s, e, _, _ in sel), 2),
                     "queues": sorted({q for _, _, q, _ in sel})}
    out["period_us"] = round((ks[hi][0] - ks[lo][0]) / 1000 / 99, 2)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1])
