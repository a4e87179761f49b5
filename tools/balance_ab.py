#!/usr/bin/env python3
"""Tile balance A/B on the GPU (rt_set_tile_balance 0 = plain grid vs 1 = adaptive): ms per frame of whole frames and
of rank 0's strip share at N ranks (interleaved 8-row strips, the row list a rank of the tiled-frame loop renders),
one stream back to back (the frame latency) and with 3 frames in flight, interleaved rounds, medians; every variant's
frame is checked equal to the first's. --variants names the arms: b0 (off), b1 (adaptive, the defaults), and b1 with
the plan's diagnostics (RT_BALANCE_SPLIT / RT_BALANCE_FRONT, read at context creation): b1s0 (no split, order
only), b1f0 (tile order, split only), b1f<k> (front class above k / 16 x the load bound), b1q<d> (extra waves for
split tiles: ntiles / d, default 8 as shipped), ...p0 (the front class's waves keep the default issue priority:
RT_BALANCE_PRIO=0), ...n0 (adaptive plans split into at most 16 parts, not 64: RT_BALANCE_FINE=0).
  python3 tools/balance_ab.py --configs C4,C2F,C2 --shares 1,4,8 --rounds 5 --variants b0,b1,b1s0"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402


def timed(c, spec, rows, bufs, streams, frames):
    W, H = spec.width, spec.height
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(streams[0])
    for k in range(frames):
        c.dispatch(W, H, bufs[k % len(bufs)], None, rows=rows, stream=streams[k % len(streams)].cuda_stream)
    if len(streams) == 1:
        e1.record(streams[0])
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / frames
    return e0.elapsed_time(e1) / frames if len(streams) == 1 else wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C4,C2F,C2,C3,C5")
    ap.add_argument("--shares", default="1,4,8")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--variants", default="b0,b1")
    a = ap.parse_args()
    variants = a.variants.split(",")
    res = {}
    for name in a.configs.split(","):
        spec = scenes.config(name)
        frames = max(4, a.frames // (8 if spec.spp > 1 else 1))
        ctxs = {}
        for v in variants:
            env = {"RT_BALANCE_SPLIT": "0" if "s0" in v else "1",
                   "RT_BALANCE_FRONT": v.split("f")[1].split("q")[0].split("p")[0].split("n")[0] if "f" in v else "8",
                   "RT_BALANCE_BUDGET": v.split("q")[1].split("p")[0].split("n")[0] if "q" in v else "8",
                   "RT_BALANCE_PRIO": "0" if "p0" in v else "1",
                   "RT_BALANCE_FINE": "0" if "n0" in v else "1"}
            os.environ.update(env)
            ctxs[v] = rt.Context(0)
            scenes.upload(ctxs[v], spec)
            ctxs[v].set_tile_balance(0 if v == "b0" else 1)
        for share in [int(x) for x in a.shares.split(",")]:
            rows = None if share == 1 else rt.strip_rows(spec.height, share, 0)
            nr = spec.height if rows is None else len(rows)
            bufs = [torch.zeros((nr, spec.width, 4), dtype=torch.uint8, device="cuda") for _ in range(3)]
            streams = [torch.cuda.Stream() for _ in range(3)]
            t = {}
            ref = None
            for rnd in range(a.rounds):
                for v in variants:
                    c = ctxs[v]
                    for key, ss in (("one", streams[:1]), ("inflight3", streams)):
                        timed(c, spec, rows, bufs, ss, 3)  # the shape's costs / plan warm
                        ms = timed(c, spec, rows, bufs, ss, frames)
                        t.setdefault(f"{v}_{key}", []).append(ms)
                    img = bufs[0].cpu().numpy()
                    if ref is None:
                        ref = img
                    assert np.array_equal(img, ref), f"{name} share {share} {v}: frame differs"
            line = {k: round(float(np.median(x)), 4) for k, x in t.items()}
            for v in variants:
                if v != "b0":
                    line[f"{v}_info"] = ctxs[v].tile_balance_info()
            res[f"{name}_N{share}"] = line
            print(name, f"share N={share}", json.dumps(line), flush=True)
        for c in ctxs.values():
            c.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "balance_ab.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
