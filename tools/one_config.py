"""Renders a few frames of one config with a given library build (for counter collection)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=rt.LIB_PATH)
ap.add_argument("--config", default="C2")
ap.add_argument("--frames", type=int, default=5)
ap.add_argument("--mode", type=int, default=-1, help="override the shade mode")
ap.add_argument("--balance", type=int, default=-1, help="rt_set_tile_balance mode (default: the context's, adaptive)")
ap.add_argument("--share", type=int, default=1, help="render rank 0's strips of a frame tiled over N ranks")
a = ap.parse_args()
spec = scenes.config(a.config)
if a.mode >= 0:
    spec.mode = a.mode
c = rt.Context(0, library=rt._load(a.lib))
scenes.upload(c, spec)
if a.balance >= 0:
    c.set_tile_balance(a.balance)
rows = rt.strip_rows(spec.height, a.share, 0) if a.share > 1 else None
out = torch.zeros((spec.height, spec.width, 4), dtype=torch.uint8, device="cuda")
for _ in range(a.frames):
    c.dispatch(spec.width, spec.height, out, rows=rows, stream=torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
print("ok")
