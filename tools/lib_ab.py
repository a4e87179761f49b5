#!/usr/bin/env python3
"""Same-box A/B of two builds of the library (e.g. a past round's, built from its commit into ab/<name>/ — package and
lib only, git-ignored — against the tree's): ms per frame with 3 frames in flight and one stream back to back,
each build in its own process, alternating (the order reversed every other round), medians over rounds.
  python3 tools/lib_ab.py --roots ab/r03,. --configs C2,C2F,C4 --rounds 3"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys, time
sys.path.insert(0, sys.argv[1])
import torch
import realtimeraytracing_gradproject_amd as rt
from realtimeraytracing_gradproject_amd import scenes
assert rt.__file__.startswith(sys.argv[1].split(":")[0]), rt.__file__
res = {}
for name in sys.argv[2].split(","):
    spec = scenes.config(name)
    c = rt.Context(0)
    scenes.upload(c, spec)
    if sys.argv[3] == "0":
        c.set_tile_balance(0)
    W, H = spec.width, spec.height
    bufs = [torch.empty((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(3)]
    ss = [torch.cuda.Stream() for _ in range(3)]
    def run(streams, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            c.dispatch(W, H, bufs[k % 3], None, stream=streams[k % len(streams)].cuda_stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / n
    n = 40 if spec.spp > 1 else 300
    run(ss, n // 4)
    res[name] = {"inflight3": run(ss, n), "one": run(ss[:1], n // 2)}
    c.close()
print(json.dumps(res))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--roots", default="ab/r03,.", help="builds; <root>:bal0 runs that build with the balance off")
    ap.add_argument("--configs", default="C2,C2F,C4")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    roots = a.roots.split(",")
    out = {}
    for rnd in range(a.rounds):
        for r in (roots if rnd % 2 == 0 else roots[::-1]):  # alternate the order: no build always runs first
            path = os.path.abspath(os.path.join(ROOT, r.split(":")[0]))
            bal = "0" if r.endswith(":bal0") else "1"
            p = subprocess.run([sys.executable, "-c", CHILD, path, a.configs, bal], capture_output=True, text=True,
                               timeout=300)
            if p.returncode != 0:
                print(p.stderr[-2000:], flush=True)
                sys.exit(1)
            res = json.loads(p.stdout.strip().splitlines()[-1])
            for cfg, v in res.items():
                for k, ms in v.items():
                    out.setdefault(cfg, {}).setdefault(f"{r}:{k}", []).append(round(ms, 4))
            print(rnd, r, json.dumps(res), flush=True)
    med = {cfg: {k: sorted(v)[len(v) // 2] for k, v in d.items()} for cfg, d in out.items()}
    print(json.dumps({"median_ms": med, "runs": out}, indent=1))


if __name__ == "__main__":
    main()
