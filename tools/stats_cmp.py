"""Traversal counters per ray of one or more library builds on the bench configs (diagnosis).

python tools/stats_cmp.py --configs C2,C4 new=path/librtamd.so pk=path/variants/pk/librtamd.so
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--configs", default="C2")
    a = ap.parse_args()
    for cfg in a.configs.split(","):
        spec = scenes.config(cfg)
        row = {}
        for v in a.variants:
            name, path = v.split("=", 1)
            c = rt.Context(0, library=rt._load(path))
            scenes.upload(c, spec)
            out = torch.zeros((spec.height, spec.width, 4), dtype=torch.uint8, device="cuda")
            c.set_stats(True)
            c.stats_reset()
            c.dispatch(spec.width, spec.height, out, stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            s = c.stats()
            rays = s["primary_rays"] + s["shadow_rays"]
            row[name] = {"rays": rays, "aabb_per_ray": round(s["aabb_tests"] / rays, 2),
                         "tri_per_ray": round(s["tri_tests"] / rays, 2),
                         "inst_per_ray": round(s["instance_entries"] / rays, 2)}
            c.close()
        print(cfg, json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
