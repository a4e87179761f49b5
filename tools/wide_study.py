#!/usr/bin/env python3
"""Runs tools/wide_study.c (design study, CPU): 4-wide vs 8-wide collapse of the same LBVH, packet
walk work of the primary and shadow packets of a single-model config.
  python3 tools/wide_study.py [--configs C2,C2F,C3] [--size 960x540]"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C2F,C3")
    ap.add_argument("--size", default="960x540")
    ap.add_argument("--treelet", type=int, default=0, help="with --sah: treelet restructuring passes instead")
    ap.add_argument("--sah", action="store_true", help="4-wide collapses of the LBVH vs a sweep-SAH binary tree over "
                                                      "the same triangles (one config per run)")
    a = ap.parse_args()
    so = "/tmp/libwide.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-ffp-contract=off", "-mfma", "-o", so,
                    os.path.join(ROOT, "tools", "wide_study.c"), "-lm", "-lpthread"], check=True)
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
        res = {}
        if a.sah:
            out = (ctypes.c_uint64 * 9)()
            assert lib.wide_study(ctypes.c_void_p(sc._h), cb, lights, w, h, 4, out) == 0
            lb = list(out)
            lib.wide_study_cost.restype = ctypes.c_double
            c0 = lib.wide_study_cost()
            assert (lib.wide_study_treelet(a.treelet) if a.treelet else lib.wide_study_sah()) == 0
            assert lib.wide_study(ctypes.c_void_p(sc._h), cb, lights, w, h, 4, out) == 0
            sa = list(out)
            print(f"{name} binary cost LBVH {c0:.1f} -> {lib.wide_study_cost():.1f}")
            for tag, o in (("LBVH", lb), ("TRLT" if a.treelet else "SAH", sa)):
                fetch = (o[0] + o[2] + o[3] + o[5]) / (lb[0] + lb[2] + lb[3] + lb[5])
                print(f"{name:4s} {tag:4s} nodes {o[8]:6d} | primary visits {o[0] / o[6]:6.2f}/pkt tri {o[2] / o[6]:5.2f}/pkt "
                      f"box {o[1] / lb[1]:.3f} | shadow visits {o[3] / o[7]:6.2f}/pkt tri {o[5] / o[7]:5.2f}/pkt "
                      f"box {o[4] / lb[4]:.3f} | fetches {fetch:.3f}", flush=True)
            continue
        for width in (4, 8):
            out = (ctypes.c_uint64 * 9)()
            assert lib.wide_study(ctypes.c_void_p(sc._h), cb, lights, w, h, width, out) == 0
            res[width] = list(out)
        for width in (4, 8):
            o = res[width]
            b = res[4]
            print(f"{name:4s} W={width} nodes {o[8]:6d} | primary: visits {o[0] / o[6]:6.2f}/pkt ({o[0] / b[0]:.3f}) "
                  f"box {o[1] / b[1]:.3f} tri {o[2] / o[6]:5.2f}/pkt | shadow: visits {o[3] / o[7]:6.2f}/pkt "
                  f"({o[3] / b[3]:.3f}) box {o[4] / b[4]:.3f} tri {o[5] / o[7]:5.2f}/pkt", flush=True)


if __name__ == "__main__":
    main()
