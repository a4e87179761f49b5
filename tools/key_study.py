#!/usr/bin/env python3
"""Runs tools/key_study.c (design study, CPU): packet fetches of whole frames per closest-hit key.
  python3 tools/key_study.py [--configs C2,C2F,C3,C4] [--size 480x270]"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KEYS = {0: "|n| (kernel)", 1: "|f|", 2: "mid-point", 3: "|n|, inside boxes by |f|"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C2F,C3,C4")
    ap.add_argument("--size", default="480x270")
    a = ap.parse_args()
    so = "/tmp/libkey.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-ffp-contract=off", "-mfma", "-o", so,
                    os.path.join(ROOT, "tools", "key_study.c"), "-lm", "-lpthread"], check=True)
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
        base = None
        img0 = None
        for k in KEYS:
            lib.set_key(k)
            o8, _, st = sc.render_spec(spec, nthreads=8, want_float=False, schedule=0)
            img0 = o8 if img0 is None else img0
            assert (o8 == img0).all(), "image must not depend on the key"
            fetch = int(st[9] + st[10] + st[11])
            base = base or fetch
            print(f"{name:4s} key {k} {KEYS[k]:28s} node {int(st[9]):9d} tri {int(st[10]):8d} fetch/base {fetch / base:.3f}",
                  flush=True)


if __name__ == "__main__":
    main()
