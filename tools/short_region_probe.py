"""Probe (diagnostics): where the fixed cost of a SHORT timed region goes (the driver runs `bench.py --steps 20
--warmup 5`: 20 frames are ~2.3 ms, so a fixed 0.1 ms is 4 %). Replays bench.py's single-rank frames-in-flight loop
on C2 (warmup, drain, synchronise, then K frames round robin over S streams) with a timing event after every frame,
and prints, relative to the host clock at t0: when the first frame's kernel started (an event recorded before it),
each frame's completion, the host issue time of the loop and the synchronise return.

  python tools/short_region_probe.py --steps 20 --warmup 5 --streams 2 --repeat 5
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--repeat", type=int, default=5)
    ap.add_argument("--gap-ms", type=float, default=0.0, help="host sleep between the warmup drain and t0")
    a = ap.parse_args()
    be = bench.make_backend(0)
    spec = scenes.config(a.config)
    be.load(spec, "packet")
    W, H = spec.width, spec.height
    streams = [be.stream() for _ in range(a.streams)]
    bufs = [be.zeros((H, W, 4)) for _ in range(a.streams)]
    # settle as bench.py does
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) < 0.3:
        for _ in range(4):
            be.dispatch(bufs[0], None, streams[0])
        be.synchronize()
    out = []
    for rep in range(a.repeat):
        for k in range(a.warmup):
            be.dispatch(bufs[k % a.streams], None, streams[k % a.streams])
        be.synchronize()
        if a.gap_ms:
            time.sleep(a.gap_ms / 1e3)
        be.synchronize()
        ev_start = be.event(True)
        evs = [be.event(True) for _ in range(a.steps)]
        h0 = time.perf_counter()
        ev_start.record(streams[0])
        for k in range(a.steps):
            s = k % a.streams
            be.dispatch(bufs[s], None, streams[s])
            evs[k].record(streams[s])
        h1 = time.perf_counter()
        be.synchronize()
        h2 = time.perf_counter()
        done = [ev_start.elapsed_time(e) for e in evs]
        out.append({"host_issue_ms": round((h1 - h0) * 1e3, 4), "wall_ms": round((h2 - h0) * 1e3, 4),
                    "gpu_last_done_ms": round(max(done), 4),
                    "per_frame_done_ms": [round(x, 4) for x in done],
                    "wall_minus_gpu_ms": round((h2 - h0) * 1e3 - max(done), 4)})
        print(json.dumps(out[-1]), flush=True)
    be.close()


if __name__ == "__main__":
    main()
