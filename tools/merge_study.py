#!/usr/bin/env python3
"""Runs tools/merge_study.c (design study, CPU): node / triangle fetches of the shadow packets when two lights' rays
share one packet (two rays per lane) against one packet per light (the kernel), for the multi-light configs.
  python3 tools/merge_study.py [--configs C4,C5] [--size 960x540]"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C4,C5")
    ap.add_argument("--size", default="960x540")
    a = ap.parse_args()
    so = "/tmp/libmerge.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-ffp-contract=off", "-mfma", "-DOPK=128", "-o", so,
                    os.path.join(ROOT, "tools", "merge_study.c"), "-lm", "-lpthread"], check=True)
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
        out = (ctypes.c_uint64 * 8)()
        assert lib.study_merge(ctypes.c_void_p(sc._h), cb, lights, len(spec.lights), w, h, out) == 0
        o = list(out)
        print(f"{name} {w}x{h} lights {len(spec.lights)}: packets {o[6]} -> {o[7]}; node fetches {o[0]} -> {o[2]} "
              f"({o[2] / o[0]:.3f}); tri fetches {o[1]} -> {o[3]} ({o[3] / max(o[1], 1):.3f}); lane box tests "
              f"{o[4]} -> {o[5]} ({o[5] / o[4]:.3f})", flush=True)


if __name__ == "__main__":
    main()
