"""Tile balance of the packet schedule (rt_set_tile_balance; VERDICT r3 #3: C4's slowest 8 x 8 tile set the frame
time). Each wave records its tile's time; a one-workgroup plan kernel splits the costliest tiles into 2 x 2 or
4 x 4 sub-packets and deals every wave longest first. The image must not depend on any of it: frames equal the
oracle's bit for bit in every layout. The forced layouts (modes 2 / 3 / 4) are deterministic, so the traversal
counters are also compared with the oracle's emulation of the same parts (oracle_render_split): every part is its
own packet with the lanes outside its sub-rectangle dead."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402

import oracle  # noqa: E402

KEYS = ["primary_rays", "shadow_rays", "aabb_tests", "tri_tests", "instance_entries", "stack_overflows"]
FETCH = ["node_fetches", "tri_fetches", "instance_fetches"]


def checked_context():
    """A context whose plan kernel verifies each work list covers every tile exactly once (RT_BALANCE_CHECK, read at
    creation; tile_balance_info()["check_bad"])."""
    os.environ["RT_BALANCE_CHECK"] = "1"
    try:
        return rt.Context(0)
    finally:
        del os.environ["RT_BALANCE_CHECK"]


def bad_tiles(a, b):
    """(tx, ty) of the 8 x 8 tiles where two frames differ (the first few), for the failure message."""
    d = (a != b).any(axis=-1)
    ys, xs = np.nonzero(d)
    return sorted({(int(x) // 8, int(y) // 8) for x, y in zip(xs, ys)})[:8], int(d.sum())


def render(c, spec, stream=None, rows=None):
    nrows = spec.height if rows is None else len(rows)
    out8 = torch.empty((nrows, spec.width, 4), dtype=torch.uint8, device="cuda")
    out32 = torch.empty((nrows, spec.width, 4), dtype=torch.float32, device="cuda")
    s = stream if stream is not None else torch.cuda.current_stream()
    c.dispatch(spec.width, spec.height, out8, out32, rows=rows, stream=s.cuda_stream)
    return out8, out32


# (config, size): one sample per pixel with 8 x 8 tiles (C4, C2F, REF's MODE 3 kernel, C1 primary only), 4 spp
# with 4 x 4-pixel tiles of 4 sample lanes each (C5), a ragged size
CASES = [("C4", (256, 136)), ("C2F", (200, 101)), ("REF", (96, 54)), ("C1", (64, 64)), ("C5", (48, 27))]


@pytest.mark.parametrize("mode", [2, 3, 4, 5])
@pytest.mark.parametrize("name,size", CASES)
def test_forced_layouts_equal_oracle_with_counters(name, size, mode):
    spec = scenes.config(name).with_size(*size)
    c = rt.Context(0)
    scenes.upload(c, spec)
    c.set_tile_balance(mode)
    c.set_stats(True)
    c.stats_reset()
    g8, g32 = render(c, spec)
    torch.cuda.synchronize()
    s = c.stats()
    o = oracle.Scene(spec)
    o8, o32, ost = o.render_spec(spec, nthreads=8, split=mode - 1)
    assert np.array_equal(g8.cpu().numpy(), o8), f"{name} mode {mode}: RGBA8"
    assert np.array_equal(g32.cpu().numpy(), o32), f"{name} mode {mode}: float"
    assert [s[k] for k in KEYS] == [int(x) for x in ost[:6]], f"{name} mode {mode}: counters"
    assert [s[k] for k in FETCH] == [int(x) for x in ost[9:12]], f"{name} mode {mode}: fetches"
    # the same layout without counters (the launch every bench frame takes)
    c.set_stats(False)
    h8, _ = render(c, spec)
    torch.cuda.synchronize()
    assert np.array_equal(h8.cpu().numpy(), o8)
    c.close()


@pytest.mark.parametrize("mode", [2, 4])
def test_forced_layouts_tile_rows_4_and_row_lists(mode):
    """8 x 4 tiles (rt_set_tile_rows(4): 4 x 2 / 2 x 1 parts) and a strip row list: images only."""
    spec = scenes.config("C4").with_size(200, 101)
    c = rt.Context(0)
    scenes.upload(c, spec)
    c.set_tile_balance(mode)
    c.set_tile_rows(4)
    o8, o32, _ = oracle.Scene(spec).render_spec(spec, nthreads=8)
    g8, g32 = render(c, spec)
    rows = rt.strip_rows(spec.height, 3, 1)
    r8, _ = render(c, spec, rows=rows)
    torch.cuda.synchronize()
    assert np.array_equal(g8.cpu().numpy(), o8) and np.array_equal(g32.cpu().numpy(), o32)
    assert np.array_equal(r8.cpu().numpy(), o8[rows])
    c.close()


@pytest.mark.parametrize("name", ["C4", "C2F"])
def test_adaptive_balance_frames_equal_oracle(name):
    """The default (adaptive) mode at the BASELINE size: the first frame records the tiles' times, the second plans
    a work list (the costliest tiles split, the long ones first) that later launches reuse, re-planned every 8
    launches into the other of the shape's two lists. Runs of frames on one stream, then on another while the first
    stream's frames still run (a list planned on one stream read on others, the next planned meanwhile, cost maps
    read while written), no synchronisation: every frame equals the oracle's; every list covered every tile
    exactly once (the plan kernel's own check); the plan ran more than once and split tiles."""
    spec = scenes.config(name)
    c = checked_context()
    scenes.upload(c, spec)
    streams = [torch.cuda.Stream() for _ in range(3)]
    order = [0] * 10 + [1] * 6 + [2] * 6 + [0] * 4
    outs = []
    for k, si in enumerate(order):
        # both outputs stay referenced until the end: a buffer dropped while its stream's kernel still writes it
        # would go to the next frame (the allocator's stream is the current one, not the kernel's)
        outs.append(render(c, spec, stream=streams[si]))
        if k == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    info = c.tile_balance_info()
    assert info["check_bad"] == 0, info
    o8, _, _ = oracle.Scene(spec).render_spec(spec, nthreads=16, want_float=False, schedule=1)
    for k, (f, _) in enumerate(outs):
        g = f.cpu().numpy()
        assert np.array_equal(g, o8), f"{name} frame {k}: tiles {bad_tiles(g, o8)} {info}"
    assert info["launches"] >= 18 and info["plans"] >= 2 and info["split"] > 0, info
    assert info["max_ticks"] > 2 * info["mean_ticks"] > 0, info
    c.close()


def test_adaptive_balance_off_for_frames_in_flight():
    """Frames in flight (each launch issued while the previous one still runs on another stream): the next frame's
    waves fill the idle slots, so the balance stays out of those launches (no cost feedback, no plan); frames equal
    the oracle's. The same shape back to back on one stream then takes it up."""
    spec = scenes.config("C4")
    c = checked_context()
    scenes.upload(c, spec)
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [render(c, spec, stream=streams[k % 3]) for k in range(12)]
    torch.cuda.synchronize()
    inflight = c.tile_balance_info()
    outs += [render(c, spec, stream=streams[0]) for _ in range(6)]
    torch.cuda.synchronize()
    single = c.tile_balance_info()
    o8, _, _ = oracle.Scene(spec).render_spec(spec, nthreads=16, want_float=False, schedule=1)
    for k, (f, _) in enumerate(outs):
        g = f.cpu().numpy()
        assert np.array_equal(g, o8), f"frame {k}: tiles {bad_tiles(g, o8)}"
    # a 1080p C4 frame runs ~0.3 ms, far longer than the host takes to issue the next: at most the first launch
    # (nothing before it) and a stray one find the previous launch done
    assert inflight["launches"] <= 3 and inflight["plans"] <= 1, inflight
    assert single["launches"] >= inflight["launches"] + 5 and single["plans"] >= 1, single
    assert single["check_bad"] == 0
    c.close()


def test_adaptive_balance_multi_frame_launch_and_off():
    """Several frames in one launch (the grid's frames share one work list) with the adaptive plan, then the plain
    grid (mode 0): every frame equals the oracle's."""
    spec = scenes.config("C4").with_size(480, 270)
    c = checked_context()
    scenes.upload(c, spec)
    comm = rt.Comm.loopback(c, 2)
    comm.set_batch(4)
    eyes = [(18.0, 14.0, 18.0), (16.0, 12.0, 20.0), (20.0, 15.0, 14.0), (17.0, 16.0, 17.0)]
    specs = []
    for e in eyes:
        sp = spec.with_size(spec.width, spec.height)
        sp.camera = (e, (0.0, 1.0, 0.0), (0.0, 1.0, 0.0))
        specs.append(sp)
    cams = np.concatenate([sp.camera_buffer().ravel() for sp in specs])
    frames = []
    for rep in range(4):
        fs = [torch.zeros((spec.height, spec.width, 4), dtype=torch.uint8, device="cuda") for _ in range(4)]
        comm.render_strips_frames(spec.width, spec.height, fs, cameras=cams)
        frames.append(fs)
    comm.synchronize()
    c.set_tile_balance(0)
    off = [torch.zeros((spec.height, spec.width, 4), dtype=torch.uint8, device="cuda") for _ in range(4)]
    comm.render_strips_frames(spec.width, spec.height, off, cameras=cams)
    comm.close()
    assert c.tile_balance_info()["check_bad"] == 0
    for q, sp in enumerate(specs):
        o8, _, _ = oracle.Scene(sp).render_spec(sp, nthreads=16, want_float=False, schedule=1)
        for rep in range(4):
            assert np.array_equal(frames[rep][q].cpu().numpy(), o8), f"launch {rep} frame {q}"
        assert np.array_equal(off[q].cpu().numpy(), o8), f"plain grid frame {q}"
    with pytest.raises(rt.RtError):
        c.set_tile_balance(6)
    c.close()


def test_refused_items_fall_back_to_the_plain_grid():
    """a work list whose parts exceed the launch's budget must not silently drop any. With a budget of
    64 extra waves (RT_BALANCE_FORCED_CAP, read at context creation) every-tile-in-16 (mode 3) cannot fit: the plan
    refuses the excess, reports it (tile_balance_info refused / refused_plans) and hands the launch the plain grid's
    list, so the frame and every traversal counter equal the oracle's plain (unsplit) packet walk. The cover check
    (RT_BALANCE_CHECK) passes on the fallback list."""
    spec = scenes.config("C4").with_size(256, 136)
    os.environ["RT_BALANCE_FORCED_CAP"] = "64"
    os.environ["RT_BALANCE_CHECK"] = "1"
    try:
        c = rt.Context(0)
    finally:
        del os.environ["RT_BALANCE_FORCED_CAP"], os.environ["RT_BALANCE_CHECK"]
    scenes.upload(c, spec)
    c.set_tile_balance(3)
    c.set_stats(True)
    c.stats_reset()
    g8, g32 = render(c, spec)
    torch.cuda.synchronize()
    s = c.stats()
    info = c.tile_balance_info()
    o8, o32, ost = oracle.Scene(spec).render_spec(spec, nthreads=8, split=0)
    assert info["refused"] > 0 and info["refused_plans"] == 1 and info["split"] == 0, info
    assert info["check_bad"] == 0, info
    assert np.array_equal(g8.cpu().numpy(), o8) and np.array_equal(g32.cpu().numpy(), o32)
    assert [s[k] for k in KEYS] == [int(x) for x in ost[:6]]
    assert [s[k] for k in FETCH] == [int(x) for x in ost[9:12]]
    c.close()


def test_split_tiles_rejoin_when_the_view_becomes_cheap():
    """a split tile's whole-wave time is not refreshed while it stays split, so the plan must judge it from
    its parts. C4 at 1080p from its own camera (a tail: the plan splits the costliest tiles, the list pays), then the
    camera turned to the sky (every ray misses: uniform, cheap tiles): within a few re-plans nothing is split and the
    list no longer pays. Every frame equals the oracle's."""
    spec = scenes.config("C4")
    sky = spec.with_size(spec.width, spec.height)
    sky.camera = ((18.0, 14.0, 18.0), (60.0, 40.0, 60.0), (0.0, 1.0, 0.0))
    c = checked_context()
    scenes.upload(c, spec)
    s = torch.cuda.Stream()
    outs = [render(c, spec, stream=s)[0] for _ in range(40)]
    torch.cuda.synchronize()
    costly = c.tile_balance_info()
    c.set_camera(sky.camera_buffer())
    outs_sky = [render(c, sky, stream=s)[0] for _ in range(80)]
    torch.cuda.synchronize()
    cheap = c.tile_balance_info()
    assert costly["pays"] == 1 and costly["split"] > 0, costly
    assert cheap["pays"] == 0 and cheap["split"] == 0 and cheap["plans"] > costly["plans"], cheap
    assert cheap["check_bad"] == 0 and cheap["refused"] == 0, cheap
    assert 0 < cheap["slots"] <= 10 * 1024, cheap  # the load bound's slots come from the runtime's occupancy
    o8, _, _ = oracle.Scene(spec).render_spec(spec, nthreads=16, want_float=False, schedule=1)
    s8, _, _ = oracle.Scene(sky).render_spec(sky, nthreads=16, want_float=False, schedule=1)
    for k in (0, 1, len(outs) - 1):
        assert np.array_equal(outs[k].cpu().numpy(), o8), f"costly frame {k}"
    for k in (0, 1, len(outs_sky) - 1):
        assert np.array_equal(outs_sky[k].cpu().numpy(), s8), f"sky frame {k}"
    c.close()


def test_load_bound_slots_match_the_hardware_residency():
    """the plan's load bound divides by the GPU's wave slots for the list's kernel. The `wavetimes`
    variant stamps every wave's start / end clock and HW_ID: a sweep over those events gives the waves resident at
    once, and it must equal rt_tile_balance_info's slots (7 waves per SIMD for these 88-SGPR kernels, not the 8 that
    hipOccupancyMaxActiveBlocksPerMultiprocessor reports). A forced layout (every tile in 4 parts,
    129,600 waves at 1080p) fills the machine many times over."""
    import os as _os
    path = _os.path.join(_os.path.dirname(rt.LIB_PATH), "variants", "wavetimes", "librtamd.so")
    c = rt.Context(0, library=rt._load(path))
    spec = scenes.config("C2")
    scenes.upload(c, spec)
    c.set_tile_balance(2)
    W, H = spec.width, spec.height
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    rec = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        c.dispatch(W, H, out, rec, stream=s)
    rec.zero_()
    c.dispatch(W, H, out, rec, stream=s)
    torch.cuda.synchronize()
    slots = c.tile_balance_info()["slots"]
    u = rec.view(torch.int32).cpu().numpy().astype(np.uint32).reshape(-1, 4)
    u = u[u[:, 1] != 0]
    assert len(u) == 4 * (W // 8) * (H // 8), len(u)  # every part's wave left its record
    t0, t1 = u[:, 0].astype(np.int64), u[:, 1].astype(np.int64)
    ev_t = np.concatenate([t0, t1])
    ev_d = np.concatenate([np.ones_like(t0), -np.ones_like(t1)])
    order = np.lexsort((ev_d, ev_t))
    peak = int(np.cumsum(ev_d[order]).max())
    assert peak == slots, (peak, slots)
    c.close()
