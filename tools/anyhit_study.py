#!/usr/bin/env python3
"""Runs tools/anyhit_study.c: shadow-packet fetches per any-hit child order (design study, CPU).
  python3 tools/anyhit_study.py [--configs C2,C2F,C4] [--size 960x540]"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ORDERS = {0: "lowest slot (kernel)", 1: "nearest entry (lead)", 2: "farthest entry (lead)",
          3: "largest area", 4: "most live rays", 5: "nearest entry, not containing origin"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C2F,C3,C4")
    ap.add_argument("--size", default="960x540")
    ap.add_argument("--orders", default="0,1,2,3,4,5")
    a = ap.parse_args()
    so = "/tmp/libanyhit.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-ffp-contract=off", "-mfma", "-o", so,
                    os.path.join(ROOT, "tools", "anyhit_study.c"), "-lm", "-lpthread"], check=True)
    import oracle
    lib = ctypes.CDLL(so)
    for n, r, args in oracle._SIGS:
        if hasattr(lib, n):
            f = getattr(lib, n)
            f.restype, f.argtypes = r, args
    oracle.lib = lib
    from realtimeraytracing_gradproject_amd import scenes
    w, h = (int(v) for v in a.size.split("x"))
    for name in a.configs.split(","):
        spec = scenes.config(name).with_size(w, h)
        sc = oracle.Scene(spec)
        cb = (ctypes.c_float * 64)(*[float(x) for x in spec.camera_buffer().ravel()])
        lights = oracle._lights(spec.lights)
        base = None
        for o in [int(x) for x in a.orders.split(",")]:
            lib.set_any_order(o)
            out = (ctypes.c_uint64 * 5)()
            lib.study_shadow(ctypes.c_void_p(sc._h), cb, lights, len(spec.lights), w, h, 0, 1, out)
            packets, nodes, tris, rays, aabb = list(out)
            base = (nodes, tris) if base is None else base
            print(f"{name:4s} order {o} {ORDERS[o]:38s} node {nodes:9d} ({nodes / base[0]:.3f}) tri {tris:9d} "
                  f"({tris / base[1]:.3f}) per packet {nodes / packets:.1f} / {tris / packets:.1f}", flush=True)


if __name__ == "__main__":
    main()
