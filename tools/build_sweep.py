"""Build time (build_ms, HIP events around the LBVH build) of random triangle soups of several sizes
for one or more library variants:  python tools/build_sweep.py base=<lib> multi=<lib> --sizes 64,1024"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import realtimeraytracing_gradproject_amd as rt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="+")
ap.add_argument("--sizes", default="2,64,256,1024,2048,4096,6320,8192")
ap.add_argument("--reps", type=int, default=15)
a = ap.parse_args()
for n in [int(x) for x in a.sizes.split(",")]:
    rng = np.random.default_rng(n)
    v = np.zeros((n * 3, 6), np.float32)
    c0 = rng.uniform(-5, 5, size=(n, 1, 3))
    v[:, :3] = (c0 + rng.uniform(-0.2, 0.2, size=(n, 3, 3))).reshape(-1, 3).astype(np.float32)
    row = [f"n={n:6d}"]
    for spec in a.variants:
        name, path = spec.split("=", 1)
        c = rt.Context(0, library=rt._load(path))
        b = c.blas_build(v)
        ms = []
        for _ in range(a.reps):
            c.blas_rebuild(b, v)
            ms.append(c.blas_info(b).build_ms)
        c.close()
        row.append(f"{name} {statistics.median(ms):.4f}")
    print("  ".join(row), flush=True)
