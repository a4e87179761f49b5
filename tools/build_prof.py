"""Rebuilds BLAS / TLAS of a config repeatedly (for rocprofv3 --kernel-trace of the LBVH build):
  python tools/build_prof.py --config C2 --reps 50
Prints build_ms (HIP events around the build kernels) per BLAS and for the TLAS."""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C2")
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--lib", default=rt.LIB_PATH)
a = ap.parse_args()
spec = scenes.config(a.config)
c = rt.Context(0, library=rt._load(a.lib))
scenes.upload(c, spec)
ms = {b: [] for b in range(len(spec.meshes))}
tl = []
for _ in range(a.reps):
    for b, (v, i) in enumerate(spec.meshes):
        c.blas_rebuild(b, v, i)
        ms[b].append(c.blas_info(b).build_ms)
    c.tlas_build([(m, x, iid, hg) for (m, x, iid, hg) in spec.instances])  # scenes.upload: BLAS id == mesh
    tl.append(c.tlas_info().build_ms)
for b in ms:
    print(f"blas {b}: prims {c.blas_info(b).prim_count} median build_ms {statistics.median(ms[b]):.4f} "
          f"min {min(ms[b]):.4f}")
print(f"tlas: median build_ms {statistics.median(tl):.4f} min {min(tl):.4f}")
c.close()
