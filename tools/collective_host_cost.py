"""Host cost per call of the collectives the strips step could use, on ONE GPU (world-1 RCCL group):
dist.gather into a list of per-rank views (bench.py's current step) vs dist.all_gather_into_tensor
into one flat buffer, for a 1080p frame's per-rank strip buffer at shares N. The GPU does almost
nothing (a world-1 collective is a local copy), so the loop time is the host's issue cost.
  python tools/collective_host_cost.py --shares 1,8
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

from realtimeraytracing_gradproject_amd import distributed as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shares", default="1,8")
    ap.add_argument("--calls", type=int, default=2000)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    comm = torch.cuda.Stream(dev)
    W, H = 1920, 1080
    out = {}
    for n in [int(x) for x in a.shares.split(",")]:
        rpr = D.padded_rows(H, n)
        local = torch.zeros((rpr, W, 4), dtype=torch.uint8, device=dev)
        gathered = torch.zeros((1, rpr, W, 4), dtype=torch.uint8, device=dev)
        parts = D.gather_parts(gathered, 1, 0)
        flat = gathered.view(-1)
        lflat = local.view(-1)

        def g():
            dist.gather(local, parts, dst=0)

        def ag():
            dist.all_gather_into_tensor(flat, lflat)

        pg = dist.distributed_c10d._get_default_group()
        gopts = dist.GatherOptions()
        gopts.rootRank = 0
        outs, ins = [parts], [local]

        def gd():  # the ProcessGroup call dist.gather makes, without its Python-side checks
            pg.gather(outs, ins, gopts).wait()

        res = {}
        for name, fn in (("gather", g), ("all_gather_into_tensor", ag), ("pg_gather", gd), ("gather", g),
                         ("all_gather_into_tensor", ag), ("pg_gather", gd)):
            with torch.cuda.stream(comm):
                for _ in range(100):
                    fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.calls):
                    fn()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
            res[name] = round((t1 - t0) / a.calls * 1e6, 2)
        out[f"share{n}"] = {"bytes": rpr * W * 4, "host_us_per_call": res}
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
