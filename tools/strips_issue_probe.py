"""Host issue cost of bench.py's strips loop on ONE GPU: bench.run_config itself, strips forced, in a
world-1 RCCL group (the gather is a local copy). (A two-thread issue variant of the loop — renders
on one host thread, gathers on another — was measured with this probe and dropped: DESIGN §7.) A frame of 1920 x (1080 / N) stands in for rank 0's share of a 1080p frame
tiled over N ranks (the same rows per rank, so the same render and issue work per step).
  python tools/strips_issue_probe.py --shares 1,8
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--shares", default="1,8")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29547")
    be = bench.HipBackend(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=be.device)
    out = {}
    for n in [int(x) for x in a.shares.split(",")]:
        base = scenes.config(a.config)
        spec = base.with_size(base.width, (base.height + n - 1) // n)
        res = {"step_ms": []}
        for _ in range(a.rounds):
            r = bench.run_config(be, spec, 1, 0, a.steps, 50, 50.0, True, True, "packet")
            res["step_ms"].append(r["tmax"] / a.steps * 1e3)
        out[f"share{n}"] = {k: round(sorted(v)[len(v) // 2], 4) for k, v in res.items()}
        out[f"share{n}"]["render_one_stream_ms"] = round(r["kernel_ms"], 4)
        out[f"share{n}"]["in_flight"] = r["in_flight"]
        print(json.dumps({f"share{n}": out[f"share{n}"]}), flush=True)
    be.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
