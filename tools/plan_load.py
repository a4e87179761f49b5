#!/usr/bin/env python3
"""The tile-balance plan under load: one library build, frames one at a time on one stream (the
balance's regime: frame latency, a rank's share) for C2F, C4 and the N = 4 share of C4, then ms per frame and the
last plan's in-kernel phase stamps (rt_tile_balance_info [12..14]). Run it under
  rocprofv3 --kernel-trace --stats -d <dir> -- python3 tools/plan_load.py --lib <librtamd.so>
for k_tile_plan's loaded duration (dispatch wait included) beside the trace kernel's; one process per build, since
the kernel names are the same in every build."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--configs", default="C2F,C4,C4/4")
    ap.add_argument("--frames", type=int, default=300)
    a = ap.parse_args()
    lib = rt._load(a.lib) if a.lib else None
    out = {"lib": a.lib or "tree"}
    for item in a.configs.split(","):
        item_, _, nst = item.partition("@")  # C2@3: frames in flight over 3 streams (the balance stays off there)
        name, _, share = item_.partition("/")
        n = int(share) if share else 1
        nstreams = int(nst) if nst else 1
        spec = scenes.config(name)
        W, H = spec.width, spec.height
        c = rt.Context(0, library=lib) if lib else rt.Context(0)
        scenes.upload(c, spec)
        rows = rt.strip_rows(H, n, 0) if n > 1 else None
        NR = len(rows) if rows is not None else H
        bufs = [torch.zeros((NR, W, 4), dtype=torch.uint8, device="cuda") for _ in range(nstreams)]
        ss = [torch.cuda.Stream() for _ in range(nstreams)]
        for k in range(60):  # clock ramp + the shape's first plans
            c.dispatch(W, H, bufs[k % nstreams], rows=rows, stream=ss[k % nstreams].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.frames):
            c.dispatch(W, H, bufs[k % nstreams], rows=rows, stream=ss[k % nstreams].cuda_stream)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.frames
        tb = c.tile_balance_info()
        out[item] = {"ms_per_frame": round(ms, 4), "plans": tb["plans"], "pays": tb["pays"], "split": tb["split"],
                     "plan_phase_us": [round(tb[k] / 100.0, 1) for k in ("plan_load_ticks", "plan_budget_ticks",
                                                                         "plan_place_ticks")]}
        c.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
