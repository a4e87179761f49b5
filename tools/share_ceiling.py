"""Strong-scaling ceilings of the tiled-frame loop, rehearsed on one GPU.

For a config and N ranks, the library's loopback communicator emulates the N-rank layout of the round-4 loop as
shipped: RGB8 strips, 4 frames per gather AND per launch (rt_render_strips_frames), the communicator's three render
streams (frames in flight), the tile balance at its default. With rt_comm_loopback_render_ranks(r, 1) only emulated
rank r renders, so one step costs this process what it costs rank r of the real run: its share's launch, the
gather copy of every rank's block into rank 0's buffer (the ncclGather's bytes, moved by a device copy instead of
xGMI) and rank 0's assembly of every frame — host issue included. The period of the real run is bounded below by
the slowest rank's share; the ceiling is the one-GPU frames loop's period (full frames, the same streams, frames in
flight: bench.py's N = 1 loop) over that. Frame time is wall clock over the whole timed region, submit -> drained,
as the reference's frame spans submit -> fence (D3D12HelloTriangle.cpp:436-470).

What the rehearsal cannot show: the xGMI transfer itself. The bytes into rank 0 per frame ((N - 1) / N of the
RGB8 frame) and the per-link rate they need at the measured ceiling are reported beside it (7 links, one per peer
on an 8-GPU node; AMD's published ~76.8 GB/s one way per link, not measured here).

  python tools/share_ceiling.py > gpurun_out/shares.jsonl     (one JSON line per (config, N, rank), then a summary)
"""
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

LINK_GBS = 76.8  # one way, per xGMI link (AMD's published 153.6 GB/s bidirectional): not measured here


def settle(ctx, spec, ms):
    """Clock ramp: full frames back to back until `ms` of wall time has passed."""
    out = torch.zeros((spec.height, spec.width, 4), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(4):
            ctx.dispatch(spec.width, spec.height, out, stream=s.cuda_stream)
        torch.cuda.synchronize()


def frames_loop(ctx, spec, frames, streams=3, rounds=3):
    """bench.py's N = 1 loop: full frames round robin over `streams` streams, each into its own buffer; best of
    `rounds` (ms per frame, wall clock, synchronised on both sides)."""
    W, H = spec.width, spec.height
    ss = [torch.cuda.Stream() for _ in range(streams)]
    bufs = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(streams)]
    best = float("inf")
    for _ in range(rounds):
        for k in range(2 * streams):
            ctx.dispatch(W, H, bufs[k % streams], stream=ss[k % streams].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(frames):
            ctx.dispatch(W, H, bufs[k % streams], stream=ss[k % streams].cuda_stream)
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) * 1e3 / frames)
    return best


def share_loop(ctx, spec, nranks, rank, frames, fpl=4, rounds=3):
    """Rank `rank`'s step of the N-rank loop (loopback, only that rank renders): ms per frame, best of `rounds`, and
    the caller's host time per call."""
    W, H = spec.width, spec.height
    comm = rt.Comm.loopback(ctx, nranks)
    comm.set_batch(fpl)
    comm.loopback_render_ranks(rank, 1)
    depth = comm.depth
    outs = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(depth)]
    ncall = [0]

    def issue(n):
        t_host = 0.0
        while n > 0:
            m = min(n, fpl)
            bufs = [outs[(ncall[0] + j) % depth] for j in range(m)]
            ncall[0] += m
            t = time.perf_counter()
            comm.render_strips_frames(W, H, bufs, None, None)
            t_host += time.perf_counter() - t
            n -= m
        return t_host

    best, host = float("inf"), float("inf")
    for _ in range(rounds):
        issue(2 * depth)
        comm.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        th = issue(frames)
        comm.synchronize()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) * 1e3 / frames)
        host = min(host, th * 1e6 / (frames / fpl))
    # where the share's period goes (rt_comm_set_phase_timing: event pairs around the render launch, the gather
    # copy, rank 0's assembly), one more pass
    comm.set_phase_timing(True)
    t0 = time.perf_counter()
    issue(frames)
    ps = comm.phase_stats()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / frames
    comm.set_phase_timing(False)
    f = max(ps["frames"], 1)
    phases = {"period_ms": round(wall, 4), "render_ms": round(ps["render_ms"] / f, 4),
              "gather_copy_ms": round(ps["gather_ms"] / f, 4), "assembly_ms": round(ps["assembly_ms"] / f, 4),
              "host_us_per_frame": round(ps["host_us"] / f, 2), "issue_thread_us_per_frame": round(ps["issue_us"] / f, 2)}
    comm.close()
    return best, host, phases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C4,C5")
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--all-ranks", action="store_true", help="every rank's share (default: rank 0 and the last)")
    ap.add_argument("--settle-ms", type=float, default=300.0)
    a = ap.parse_args()
    frames_of = {"C2": 400, "C2F": 400, "C3": 400, "C4": 200, "C5": 24}
    for name in a.configs.split(","):
        spec = scenes.config(name)
        ctx = rt.Context(0)
        scenes.upload(ctx, spec)
        settle(ctx, spec, a.settle_ms)
        nf = frames_of.get(name, 200)
        one = frames_loop(ctx, spec, nf)
        rgb_frame = spec.width * spec.height * 3
        print(json.dumps({"config": name, "n": 1, "ms_per_frame": round(one, 4), "loop": "frames, 3 streams"}),
              flush=True)
        for n in [int(x) for x in a.ranks.split(",")]:
            ranks = range(n) if a.all_ranks else sorted({0, n - 1})
            per = {}
            for r in ranks:
                ms, host, phases = share_loop(ctx, spec, n, r, nf)
                per[r] = ms
                print(json.dumps({"config": name, "n": n, "rank": r, "ms_per_frame": round(ms, 4),
                                  "host_us_per_call": round(host, 2), "frames": nf, "frames_per_launch": 4,
                                  "frames_per_gather": 4, "phases": phases}), flush=True)
            worst = max(per.values())
            ingress = rgb_frame * (n - 1) / n  # bytes into rank 0 per frame
            print(json.dumps({
                "config": name, "n": n, "summary": True, "one_gpu_ms": round(one, 4),
                "rank0_ms": round(per[0], 4), "slowest_share_ms": round(worst, 4),
                "ceiling_x": round(one / worst, 2), "target_x": 6.0 if n == 8 else None,
                "ingress_bytes_per_frame": int(ingress),
                "ingress_gbs_at_ceiling": round(ingress / (worst * 1e-3) / 1e9, 1),
                "per_link_gbs_at_ceiling": round(ingress / (worst * 1e-3) / 1e9 / (n - 1), 1),
                "per_link_frac_of_76.8": round(ingress / (worst * 1e-3) / 1e9 / (n - 1) / LINK_GBS, 3)}),
                flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
