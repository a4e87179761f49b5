#!/usr/bin/env python3
"""What a small kernel on a second stream waits for while trace frames run (k_tile_plan's
loaded duration is ~2x its in-kernel phase stamps). One-stream C4 frames back to back; every 8th frame a tiny torch
kernel (one workgroup: x.add_(1) on 64 floats) goes on a second stream, and a 1,024-thread, LDS-heavy one (a torch
sum over 256 K floats) on a third. Under rocprofv3 --kernel-trace their durations against the same kernels on an
idle GPU say whether the wait is for resources (wave slots / LDS on one CU) or for the queue's turn.
  rocprofv3 --kernel-trace --stats -d <dir> -- python3 tools/queue_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402


def main():
    spec = scenes.config("C4")
    c = rt.Context(0)
    scenes.upload(c, spec)
    c.set_tile_balance(0)  # no plans of our own: only the probe kernels beside the frames
    W, H = spec.width, spec.height
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    s_main, s_small, s_big = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    small = torch.zeros(64, device="cuda")
    big = torch.ones(1 << 18, device="cuda")
    res = torch.zeros(1, device="cuda")
    import ctypes
    probe = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "libdispatch_probe.so"))
    probe.dispatch_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    pout = torch.zeros(4, dtype=torch.int32, device="cuda")
    s_probe = [torch.cuda.Stream() for _ in range(4)]

    def probes():
        with torch.cuda.stream(s_small):
            small.add_(1.0)
        with torch.cuda.stream(s_big):
            torch.sum(big, dim=0, out=res)
        for kind in range(4):  # the plan's shape (1024 threads, 135 KB LDS), and without each of the two
            assert probe.dispatch_probe(kind, pout.data_ptr(), s_probe[kind].cuda_stream) == 0
    torch.cuda.synchronize()
    # idle reference: the probe kernels alone
    for _ in range(20):
        probes()
        torch.cuda.synchronize()
    # loaded: beside back-to-back frames
    for k in range(400):
        c.dispatch(W, H, out, stream=s_main.cuda_stream)
        if k % 8 == 4:
            probes()
    torch.cuda.synchronize()
    c.close()
    print("ok")


if __name__ == "__main__":
    main()
