#!/usr/bin/env python3
"""Runs tools/shadow_study.c (design study, CPU): per-wave node / triangle fetches of the shadow
packets under several regroupings of the same shadow rays, for the LAMBERT_SHADOW configs.
  python3 tools/shadow_study.py [--configs C2,C4,C5] [--size 960x540] [--group 2]
Prints one line per (config, mode). The cost unit of the packet walk is a per-wave fetch (one
scalar load + 64 lanes of slab / Moller-Trumbore VALU), so fewer fetches = less work."""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MODES = {0: "per wave, per light (kernel)", 1: "per wave, lights compacted", 2: "G waves, per light compacted",
         3: "G waves, lights compacted", 4: "per wave, per light, sorted by instance",
         5: "G waves, per light, sorted by instance", 6: "G waves, per light, sorted by origin Morton",
         7: "frame, per light, sorted by instance, Morton", 8: "frame, per light, sorted by origin Morton"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C4,C5")
    ap.add_argument("--size", default="960x540")
    ap.add_argument("--group", type=int, default=2)
    ap.add_argument("--modes", default="0,1,2,3,4,5,6")
    a = ap.parse_args()
    so = "/tmp/libstudy.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-ffp-contract=off", "-mfma", "-o", so,
                    os.path.join(ROOT, "tools", "shadow_study.c"), "-lm", "-lpthread"], check=True)
    import oracle
    lib = ctypes.CDLL(so)
    for n, r, args in oracle._SIGS:
        if not hasattr(lib, n):  # the raster oracle is not part of the study build
            continue
        f = getattr(lib, n)
        f.restype, f.argtypes = r, args
    lib.study_shadow.restype = ctypes.c_int
    oracle.lib = lib  # Scene() below lives in the study library
    from realtimeraytracing_gradproject_amd import scenes
    w, h = (int(v) for v in a.size.split("x"))
    for name in a.configs.split(","):
        spec = scenes.config(name).with_size(w, h)
        sc = oracle.Scene(spec)
        cb = (ctypes.c_float * 64)(*[float(x) for x in spec.camera_buffer().ravel()])
        lights = oracle._lights(spec.lights)
        base = None
        for m in [int(x) for x in a.modes.split(",")]:
            out = (ctypes.c_uint64 * 5)()
            lib.study_shadow(ctypes.c_void_p(sc._h), cb, lights, len(spec.lights), w, h, m, a.group, out)
            packets, nodes, tris, rays, aabb = list(out)
            cost = nodes + tris
            base = cost if base is None else base
            print(f"{name:4s} mode {m} {MODES[m]:45s} packets {packets:8d} rays {rays:9d} node {nodes:9d} "
                  f"tri {tris:9d} fetch/base {cost / base:.3f} rays/packet {rays / max(packets, 1):.1f}", flush=True)


if __name__ == "__main__":
    main()
