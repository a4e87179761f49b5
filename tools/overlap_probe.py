"""Frames in flight: K frames of a config rendered back to back on ONE stream (each launch waits
for the previous) vs alternating over S streams into S buffers (frame k + 1's waves fill the
wave slots frame k's tail leaves idle). Whole-loop wall time per frame, interleaved rounds.
  python tools/overlap_probe.py --config C2 --shares 1,8 --streams 2
"""
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
    ap.add_argument("--config", default="C2")
    ap.add_argument("--shares", default="1,8")
    ap.add_argument("--streams", default="2,3")
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--lib", default="", help="a library variant (tools/build_variant.sh) instead of the shipped one")
    a = ap.parse_args()
    spec = scenes.config(a.config)
    W, H = spec.width, spec.height
    ctx = rt.Context(0, library=rt._load(a.lib)) if a.lib else rt.Context(0)
    scenes.upload(ctx, spec)
    out = {}
    for n in [int(x) for x in a.shares.split(",")]:
        rows = rt.strip_rows(H, n, 0) if n > 1 else None
        NR = len(rows) if rows is not None else H
        variants = [1] + [int(x) for x in a.streams.split(",")]
        streams = {v: [torch.cuda.Stream() for _ in range(v)] for v in variants}
        bufs = {v: [torch.empty((NR, W, 4), dtype=torch.uint8, device="cuda") for _ in range(v)] for v in variants}
        res = {v: [] for v in variants}
        for v in variants:  # warm
            for k in range(50):
                ctx.dispatch(W, H, bufs[v][k % v], None, rows=rows, stream=streams[v][k % v].cuda_stream)
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for v in variants:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(a.frames):
                    ctx.dispatch(W, H, bufs[v][k % v], None, rows=rows, stream=streams[v][k % v].cuda_stream)
                torch.cuda.synchronize()
                res[v].append((time.perf_counter() - t0) / a.frames * 1e3)
        out[f"share{n}"] = {f"streams{v}": round(sorted(x)[len(x) // 2], 4) for v, x in res.items()}
        print(json.dumps({f"share{n}": out[f"share{n}"]}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
