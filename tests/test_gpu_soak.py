"""Soak: long runs of the adaptive tile balance with the camera moving every frame (the async plan / list swap, the
cost maps written and read by launches on several streams, split tiles rejoining as the view changes),
alternating segments of one-at-a-time frames (the balance active: feedback, plans, lists) and frames in flight over
three streams (the balance off, then taken up again). Every frame gets its own camera; a sample of frames spread over
the run is compared with the oracle bit for bit, and the plan kernel's own cover check (RT_BALANCE_CHECK) must never
have failed."""
import json
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402

import oracle  # noqa: E402


def orbit(spec, k, n):
    """Frame k of n on a circle around the scene's target, the height swinging (views from grazing to steep)."""
    (ex, ey, ez), tgt, up = spec.camera
    r = math.hypot(ex - tgt[0], ez - tgt[2])
    a = math.atan2(ez - tgt[2], ex - tgt[0]) + 2.0 * math.pi * k / n
    h = ey * (0.55 + 0.45 * math.cos(5.0 * math.pi * k / n))
    sp = spec.with_size(spec.width, spec.height)
    sp.camera = ((tgt[0] + r * math.cos(a), h, tgt[2] + r * math.sin(a)), tgt, up)
    return sp


@pytest.mark.parametrize("name,size", [("C2F", (640, 360)), ("C4", (640, 360))])
def test_balance_soak_moving_camera(name, size):
    base = scenes.config(name).with_size(*size)
    os.environ["RT_BALANCE_CHECK"] = "1"
    try:
        c = rt.Context(0)
    finally:
        del os.environ["RT_BALANCE_CHECK"]
    scenes.upload(c, base)
    W, H = size
    streams = [torch.cuda.Stream() for _ in range(3)]
    n = 360
    outs, specs = [], []
    for k in range(n):
        seg = (k // 60) % 2  # 0: one stream (balance active), 1: three streams in flight
        sp = orbit(base, k, n)
        c.set_camera(sp.camera_buffer())
        out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
        c.dispatch(W, H, out, stream=streams[0 if seg == 0 else k % 3].cuda_stream)
        outs.append(out)
        specs.append(sp)
    torch.cuda.synchronize()
    info = c.tile_balance_info()
    assert info["check_bad"] == 0 and info["refused"] == 0, info
    assert info["plans"] >= 1, info
    # the re-plan cadence of balance_wants_plan, over the shape's active launches: a list that pays is
    # re-planned every 8 of them once the previous plan has landed. At 640 x 360 a frame takes 15-40 us and a plan
    # ~100 us beside them (its dispatch waits for a CU with 16 free wave slots), so a plan lands 3-7
    # launches after it starts; the three-stream segments also count active launches that cannot start a plan
    # (active_run resets). Measured: C2F 6 plans over 181 active launches. So a paying list is re-planned at least
    # every 64; a list that does not pay re-checks every 32 (a tail splitting could not shorten) or 128 launches (no
    # tail, or coherent tiles), doubling after each further plan that did not pay — never more often than every 32
    act = info["launches"]
    print(name, json.dumps(info))
    if info["pays"]:
        assert info["plans"] >= act // 64, json.dumps(info)
    else:
        assert info["plans"] <= 2 + act // 32, json.dumps(info)
    o = oracle.Scene(base)
    for k in range(0, n, 15):
        want, _, _ = o.render_spec(specs[k], nthreads=16, want_float=False)
        got = outs[k].cpu().numpy()
        bad = int((got != want).any(axis=2).sum())
        assert bad == 0, f"{name} frame {k}: {bad} pixels differ ({info})"
    c.close()


def test_balance_replans_every_8_launches_while_it_pays():
    """the cadence pinned where the list pays. C4 at 1920 x 1080, one frame at a time with the camera
    orbiting (each view changes which tiles are costly), the host waiting for each frame as the reference does
    (WaitForPreviousFrame, D3D12HelloTriangle.cpp:627-647): the slowest tiles outlast the load bound, so every plan
    splits some and pays, and balance_wants_plan re-plans every kReplan = 8 active launches (the plan lands before the
    next launch): over 160 launches at least 160 / 16 plans, each list a valid cover (RT_BALANCE_CHECK). (A host that
    issues far ahead of the GPU sees a plan land only when the GPU reaches it, so its cadence counts in launches the
    GPU has run, not launches issued: the soak above.)"""
    base = scenes.config("C4")
    os.environ["RT_BALANCE_CHECK"] = "1"
    try:
        c = rt.Context(0)
    finally:
        del os.environ["RT_BALANCE_CHECK"]
    scenes.upload(c, base)
    W, H = base.width, base.height
    s = torch.cuda.Stream()
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    n = 160
    for k in range(n):
        c.set_camera(orbit(base, k, 4 * n).camera_buffer())
        c.dispatch(W, H, out, stream=s.cuda_stream)
        s.synchronize()  # the frame's fence
    torch.cuda.synchronize()
    info = c.tile_balance_info()
    assert info["check_bad"] == 0 and info["refused"] == 0, info
    print(json.dumps(info))
    assert info["launches"] == n and info["pays"] == 1, json.dumps(info)
    assert info["plans"] >= n // 16, json.dumps(info)
    want, _, _ = oracle.Scene(base).render_spec(orbit(base, n - 1, 4 * n), nthreads=16, want_float=False)
    assert int((out.cpu().numpy() != want).any(axis=2).sum()) == 0
    c.close()


def test_loopback_loop_soak_moving_camera():
    """The tiled multi-GPU loop (loopback, N = 4, 4 frames per gather and per launch) over 160 frames with a camera
    each: sampled frames equal the oracle's."""
    base = scenes.config("C4").with_size(480, 270)
    c = rt.Context(0)
    scenes.upload(c, base)
    comm = rt.Comm.loopback(c, 4)
    comm.set_batch(4)
    W, H = base.width, base.height
    n = 160
    frames, specs = [], []
    for k0 in range(0, n, 4):
        sps = [orbit(base, k, n) for k in range(k0, k0 + 4)]
        fs = [torch.empty((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(4)]
        comm.render_strips_frames(W, H, fs, cameras=np.concatenate([sp.camera_buffer().ravel() for sp in sps]))
        frames += fs
        specs += sps
    comm.synchronize()
    comm.close()
    o = oracle.Scene(base)
    for k in range(0, n, 13):
        want, _, _ = o.render_spec(specs[k], nthreads=16, want_float=False)
        bad = int((frames[k].cpu().numpy() != want).any(axis=2).sum())
        assert bad == 0, f"frame {k}: {bad} pixels differ"
    c.close()
