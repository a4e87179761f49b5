"""Probe (diagnostics, one GPU, world-1 RCCL): does splitting the strips loop over TWO communicators raise the step
rate where the host issue binds (a rank's share at N = 8)? Frames alternate between the communicators, each with
its own gather stream, issue thread and render stream(s); the gathers of one communicator stay in frame order, so
the collective order is the same on every rank. Reported: ms per frame once drained, best of `rounds`.

  python tools/dual_comm_probe.py --size 1920x136 --frames 400
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--size", default="1920x136")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    spec = scenes.config(a.config)
    if a.size:
        spec = spec.with_size(*(int(v) for v in a.size.lower().split("x")))
    W, H = spec.width, spec.height
    ctx = rt.Context(0)
    scenes.upload(ctx, spec)

    def run(comms, frames_per):
        calls = [0] * len(comms)
        bufs = [[torch.zeros((H, W, 4), dtype=torch.uint8, device=dev) for _ in range(c.depth)] for c in comms]

        def step(k):
            i = k % len(comms)
            c = comms[i]
            c.render_strips(W, H, bufs[i][calls[i] % c.depth], None)
            calls[i] += 1

        def sync():
            for c in comms:
                c.synchronize()
            torch.cuda.synchronize()

        best, issue = float("inf"), float("inf")
        for _ in range(a.rounds):
            for k in range(40):
                step(k)
            sync()
            t0 = time.perf_counter()
            for k in range(frames_per):
                step(k)
            t1 = time.perf_counter()
            sync()
            t2 = time.perf_counter()
            best = min(best, (t2 - t0) * 1e3 / frames_per)
            issue = min(issue, (t1 - t0) * 1e6 / frames_per)
        return {"ms_per_frame": round(best, 4), "host_issue_us_per_step": round(issue, 2),
                "depths": [c.depth for c in comms]}

    out = {"config": a.config, "size": f"{W}x{H}", "frames": a.frames}
    variants = [("one_comm_3slots", 1, "3"), ("two_comms_1slot", 2, "1"), ("two_comms_2slots", 2, "2"),
                ("three_comms_1slot", 3, "1")]
    for name, n, slots in variants:
        os.environ["RT_COMM_SLOTS"] = slots
        comms = [rt.Comm(ctx, 1, 0, rt.comm_unique_id()) for _ in range(n)]
        out[name] = run(comms, a.frames)
        for c in comms:
            c.close()
        print(json.dumps({name: out[name]}), file=sys.stderr, flush=True)
    os.environ.pop("RT_COMM_SLOTS", None)
    ctx.close()
    dist.destroy_process_group()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
