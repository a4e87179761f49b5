"""The N > 1 layout of the native multi-GPU frame loop (rt_comm_*, rt_render_strips) on
one GPU, through the library's loopback transport (rt_comm_init_loopback): this process renders every emulated
rank's interleaved strips into that rank's block of a pipeline slot, and the "gather" is a device copy into rank 0's
rank-major buffer issued where ncclGather is. Plan, frame batching (one gather per b frames, frame b at b frames
into each rank's block, the rank-strided RGB8 -> RGBA8 assembly), events and tails are the RCCL path's. Every
assembled frame equals the oracle's frame of the reference's DispatchRays W x H (D3D12HelloTriangle.cpp:584-592)
bit for bit, with a camera change per frame."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402

import oracle  # noqa: E402

# C2 (the BASELINE frame) and a ragged frame: 1083 rows = 135 full 8-row strips + a 3-row one, which leaves the
# ranks with different row counts (some a strip short) at N = 2, 3 and 8; then one small frame per assembly kernel
# (launch_assemble_frames): width a multiple of 16 (16 pixels per thread), of 4 only (4 per thread), neither (generic)
SIZES = [(1920, 1080), (1920, 1083), (208, 97), (200, 101), (202, 99)]
SIZE_IDS = ["1920x1080", "1920x1083", "208x97", "200x101", "202x99"]
EYES = [(1.5, 1.5, 1.5), (2.2, 1.4, 1.1), (1.1, 1.9, 2.4), (3.0, 2.0, 0.5)]  # the first is the reference camera
_ORACLE = {}


def _spec(size, k):
    sp = scenes.config("C2").with_size(*size)
    sp.camera = (EYES[k], (0.0, 0.0, 0.0), (0.0, 1.0, 0.0))
    return sp


def _oracle_frame(size, k):
    key = (size, k)
    if key not in _ORACLE:
        sp = _spec(size, k)
        o8, _, _ = oracle.Scene(sp).render_spec(sp, nthreads=16, want_float=False, schedule=1)
        _ORACLE[key] = o8
    return _ORACLE[key]


def _check(frames, size, cams, what):
    for k, f in enumerate(frames):
        got = f.cpu().numpy()
        want = _oracle_frame(size, cams[k])
        bad = int((got != want).any(axis=2).sum())
        assert bad == 0, f"{what}: frame {k} (camera {cams[k]}): {bad} pixels differ"


@pytest.mark.parametrize("size", SIZES, ids=SIZE_IDS)
@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_loopback_strips_every_batch_equals_oracle(size, nranks):
    """N ranks x frames per gather 1, 2, 4: 2 x depth + 1 frames (every slot reused, the last batch partly filled
    and gathered as it is at rt_comm_synchronize), a camera change per frame, each frame into its own buffer, the
    library's own render streams (frames in flight)."""
    W, H = size
    c = rt.Context(0)
    scenes.upload(c, _spec(size, 0))
    for batch in (1, 2, 4):
        comm = rt.Comm.loopback(c, nranks)
        comm.set_batch(batch)
        assert comm.batch == batch
        n = 2 * comm.depth + 1
        frames = [torch.full((H, W, 4), 7, dtype=torch.uint8, device="cuda") for _ in range(n)]
        cams = [k % len(EYES) for k in range(n)]
        for k in range(n):
            c.set_camera(_spec(size, cams[k]).camera_buffer())
            comm.render_strips(W, H, frames[k], None)
        comm.synchronize()
        _check(frames, size, cams, f"N={nranks} batch={batch}")
        comm.close()
    c.close()


@pytest.mark.parametrize("nranks", [2, 8])
def test_loopback_frames_in_one_launch_equal_oracle(nranks):
    """rt_render_strips_frames: b frames, one camera each, rendered by ONE launch per rank into one slot (grid z =
    frame), one gather; calls of 4, 3 (a new slot after the 4), 1 and 2 frames at batch 4, on a caller stream."""
    size = (1920, 1083)
    W, H = size
    c = rt.Context(0)
    scenes.upload(c, _spec(size, 0))
    comm = rt.Comm.loopback(c, nranks)
    comm.set_batch(4)
    stream = torch.cuda.Stream()
    frames, cams = [], []
    k = 0
    for nf in (4, 3, 1, 2, 4):
        fs = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(nf)]
        cs = [(k + j) % len(EYES) for j in range(nf)]
        cb = np.concatenate([_spec(size, q).camera_buffer().ravel() for q in cs])
        comm.render_strips_frames(W, H, fs, cameras=cb, stream=stream.cuda_stream)
        frames += fs
        cams += cs
        k += nf
    comm.synchronize()
    _check(frames, size, cams, f"N={nranks} frames-per-launch")
    with pytest.raises(rt.RtError):  # more frames than a slot holds
        comm.render_strips_frames(W, H, [frames[0]] * 5)
    comm.close()
    c.close()


# The multi-GPU configs through the same loop: the workloads the 8-GPU run tiles first. C5 is 4 spp
# (the KS = 2 sample-lane kernel: a wave covers 4 x 4 pixels, RayGen.hlsl:33's pixel mapping per sample) over 257
# instances, C4 64 instances and 2 lights. Eyes: the config's own first, then moves around the grid.
GRID_EYES = {"C4": [(18.0, 14.0, 18.0), (15.0, 12.0, 21.0), (21.0, 16.0, 14.0), (-17.0, 13.0, 19.0)],
             "C5": [(30.0, 22.0, 30.0), (26.0, 18.0, 34.0), (34.0, 26.0, 25.0), (-28.0, 20.0, 31.0)]}
_GRID_ORACLE = {}


def _grid_spec(name, size, k):
    sp = scenes.config(name).with_size(*size)
    _, at, up = sp.camera
    sp.camera = (GRID_EYES[name][k], at, up)
    return sp


def _grid_oracle(name, size, k):
    key = (name, size, k)
    if key not in _GRID_ORACLE:
        sp = _grid_spec(name, size, k)
        _GRID_ORACLE[key] = oracle.Scene(sp).render_spec(sp, nthreads=16, want_float=False, schedule=1)[0]
    return _GRID_ORACLE[key]


@pytest.mark.parametrize("name,size,nranks,calls", [
    ("C5", (960, 540), 8, (4, 4, 3)),      # 540 rows: 67.5 strips over 8 ranks (ragged), the last batch 3 of 4
    ("C5", (3840, 2160), 8, (1,)),         # one full BASELINE frame (configs[4]), a batch of 1 of 4
    ("C4", (1920, 1080), 4, (4, 4, 2)),    # BASELINE configs[3] at its N = 4
], ids=["C5-960x540-N8", "C5-3840x2160-N8", "C4-1920x1080-N4"])
def test_loopback_multisample_and_grid_frames_equal_oracle(name, size, nranks, calls):
    """rt_render_strips_frames at 4 frames per gather and up to 4 frames per launch (one camera each, grid z =
    frame) on the communicator's own render streams, the tile balance at its default: every assembled frame of
    C5 (4 spp, N = 8) and C4 (N = 4) equals the oracle's, the last batch partly filled and gathered at
    rt_comm_synchronize."""
    W, H = size
    c = rt.Context(0)
    scenes.upload(c, _grid_spec(name, size, 0))
    comm = rt.Comm.loopback(c, nranks)
    comm.set_batch(4)
    neyes = len(GRID_EYES[name])
    frames, cams, k = [], [], 0
    for nf in calls:
        fs = [torch.full((H, W, 4), 7, dtype=torch.uint8, device="cuda") for _ in range(nf)]
        cs = [(k + j) % neyes for j in range(nf)]
        cb = np.concatenate([_grid_spec(name, size, q).camera_buffer().ravel() for q in cs])
        comm.render_strips_frames(W, H, fs, cameras=cb, stream=None)
        frames += fs
        cams += cs
        k += nf
    comm.synchronize()
    for f, q in zip(frames, cams):
        got = f.cpu().numpy()
        bad = int((got != _grid_oracle(name, size, q)).any(axis=2).sum())
        assert bad == 0, f"{name} {W}x{H} N={nranks}: camera {q}: {bad} pixels differ"
    comm.close()
    c.close()


@pytest.mark.parametrize("loop", ["loopback8", "rccl1"])
def test_close_with_partly_filled_batch_returns(loop):
    """rt_comm_destroy with a partly filled slot and no rt_comm_synchronize: 2 frames at 3
    frames per gather, then close(). The destroy drains the slot through the issue thread before stopping it, so it
    returns (the test runs under pytest's timeout) and both frames are complete and correct."""
    size = (960, 544)
    W, H = size
    c = rt.Context(0)
    scenes.upload(c, _spec(size, 0))
    comm = rt.Comm.loopback(c, 8) if loop == "loopback8" else rt.Comm(c, 1, 0, rt.comm_unique_id())
    comm.set_batch(3)
    frames = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)]
    cams = [1, 2]
    for k in range(2):
        c.set_camera(_spec(size, cams[k]).camera_buffer())
        comm.render_strips(W, H, frames[k], None)
    comm.close()  # no synchronize
    torch.cuda.synchronize()
    _check(frames, size, cams, f"{loop} close()")
    c.close()


def test_later_frames_on_other_streams_are_ordered():
    """A slot's later frames issued on other streams than its first: each frame's render waits for the
    work already queued on its own stream, and its tail comes back to that stream. Each frame's stream first fills
    the frame buffer with a pattern (queued, not synchronised) and the render must come after it; then that stream
    alone is synchronised and must see its assembled frame."""
    size = (640, 360)
    W, H = size
    c = rt.Context(0)
    scenes.upload(c, _spec(size, 0))
    comm = rt.Comm.loopback(c, 3)
    comm.set_batch(3)
    streams = [torch.cuda.Stream() for _ in range(3)]
    frames = [torch.empty((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(3)]
    cams = [0, 3, 2]
    for k in range(3):
        with torch.cuda.stream(streams[k]):
            torch.cuda._sleep(2_000_000)  # keeps the stream busy, so an unordered render would run first
            frames[k].fill_(9)
        c.set_camera(_spec(size, cams[k]).camera_buffer())
        comm.render_strips(W, H, frames[k], streams[k].cuda_stream)
    torch.cuda.ExternalStream(comm.stream).synchronize()  # the slot is gathered and its tails issued
    for k in (2, 1, 0):
        streams[k].synchronize()
        _check([frames[k]], size, [cams[k]], f"stream {k}")
    comm.close()
    c.close()


def test_forget_stream_then_tlas_update():
    """rt_forget_stream: a stream that launched frames is destroyed; the next rt_tlas_build(update_only) must not
    record on it. The communicator's own render streams go through the same path at rt_comm_destroy."""
    spec = scenes.config("C2F").with_size(256, 144)
    c = rt.Context(0)
    scenes.upload(c, spec)
    out = torch.zeros((spec.height, spec.width, 4), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    c.dispatch(spec.width, spec.height, out, stream=s.cuda_stream)
    c.forget_stream(s.cuda_stream)
    comm = rt.Comm.loopback(c, 2)
    comm.render_strips(spec.width, spec.height, out, None)
    comm.close()  # its render streams read the TLAS: forgotten before they are destroyed
    torch.cuda.synchronize()
    del s
    inst = [(m, x, iid, hg) for (m, x, iid, hg) in spec.instances]
    for _ in range(3):
        c.tlas_build(inst, update_only=True)
    c.dispatch(spec.width, spec.height, out, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    o8, _, _ = oracle.Scene(spec).render_spec(spec, nthreads=16, want_float=False, schedule=1)
    assert np.array_equal(out.cpu().numpy(), o8)
    c.close()


@pytest.mark.parametrize("loop", ["loopback8", "rccl1"])
def test_abort_with_partly_filled_batch_returns(loop):
    """rt_comm_abort, the failure path: 2 frames at 3 frames per gather, then abort() — no drain,
    no further collective (a real peer may never call again), ncclCommAbort for RCCL. It returns under the test
    timeout, and the context keeps rendering correct frames, also through a new communicator."""
    size = (960, 544)
    W, H = size
    c = rt.Context(0)
    scenes.upload(c, _spec(size, 0))
    comm = rt.Comm.loopback(c, 8) if loop == "loopback8" else rt.Comm(c, 1, 0, rt.comm_unique_id())
    comm.set_batch(3)
    frames = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)]
    for k in range(2):
        c.set_camera(_spec(size, k + 1).camera_buffer())
        comm.render_strips(W, H, frames[k], None)
    comm.abort()
    comm.abort()  # a second abort (or close) of the same Python object is a no-op
    comm.close()
    torch.cuda.synchronize()
    c.set_camera(_spec(size, 3).camera_buffer())
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    c.dispatch(W, H, out, stream=torch.cuda.current_stream().cuda_stream)
    comm2 = rt.Comm.loopback(c, 2)
    again = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    comm2.render_strips(W, H, again, None)
    comm2.close()
    torch.cuda.synchronize()
    _check([out, again], size, [3, 3], f"{loop} after abort")
    c.close()


def test_unclosed_communicator_garbage_collected(recwarn):
    """a loopback communicator dropped unclosed drains like close() — the frames already handed to
    render_strips (2 of a 3-frame batch) are rendered and assembled; an RCCL one aborts (peers may never match a
    draining gather) and warns that it discarded pending frames."""
    import gc
    size = (960, 544)
    W, H = size
    c = rt.Context(0)
    scenes.upload(c, _spec(size, 0))
    comm = rt.Comm.loopback(c, 8)
    comm.set_batch(3)
    frames = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()  # the zero fill (torch's stream) before the communicator's own streams write
    for k in range(2):
        c.set_camera(_spec(size, k + 1).camera_buffer())
        comm.render_strips(W, H, frames[k], None)
    del comm
    gc.collect()
    torch.cuda.synchronize()
    _check(frames, size, [1, 2], "loopback dropped unclosed")
    assert not [w for w in recwarn if issubclass(w.category, ResourceWarning)]
    comm = rt.Comm(c, 1, 0, rt.comm_unique_id())
    comm.set_batch(3)
    comm.render_strips(W, H, frames[0], None)
    with pytest.warns(ResourceWarning, match="close"):
        comm.__del__()
    del comm
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    c.set_camera(_spec(size, 3).camera_buffer())
    c.dispatch(W, H, out, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    _check([out], size, [3], "after the RCCL abort")
    c.close()


def test_many_emulated_ranks_never_synchronise_the_device():
    """every emulated rank's row list is its own tile-balance shape, so 40 ranks exceed the context's table
    of cost maps. A full table must not cost a device-wide synchronisation per launch (it used to evict with
    hipDeviceSynchronize on every rank's dispatch): the launches that find no idle map run the plain grid. Over
    steady-state frames the context's device-sync counter does not move, and every frame equals the oracle's."""
    size = (1920, 1080)
    W, H = size
    c = rt.Context(0)
    scenes.upload(c, _spec(size, 0))
    comm = rt.Comm.loopback(c, 40)
    comm.set_batch(2)
    frames = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(comm.depth)]
    for k in range(comm.depth):  # warm: plans, slots, the cost maps
        comm.render_strips(W, H, frames[k], None)
    comm.synchronize()
    before = c.counters()
    cams = []
    for k in range(2 * comm.depth):
        q = k % len(EYES)
        c.set_camera(_spec(size, q).camera_buffer())
        comm.render_strips(W, H, frames[k % comm.depth], None)
        cams.append(q)
    comm.synchronize()
    after = c.counters()
    assert after["device_syncs"] == before["device_syncs"], (before, after)
    assert after["balance_maps"] <= 32 and after["balance_full"] + after["balance_recycled"] > 0, after
    _check(frames, size, cams[-comm.depth:], "40 emulated ranks")
    comm.close()
    c.close()
