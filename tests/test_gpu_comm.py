"""The native multi-GPU frame loop (rt_comm_* / rt_render_strips) on the GPU box: a world-1 RCCL
communicator (a one-GPU box cannot host two RCCL ranks). Frames rendered through render -> ncclGather ->
rt_assemble_strips, several in flight on different streams, equal the oracle's bit for bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402

import oracle  # noqa: E402


def test_render_strips_world1_equals_oracle():
    spec = scenes.config("C2")  # the headline frame, full 1080p
    c = rt.Context(0)
    scenes.upload(c, spec)
    comm = rt.Comm(c, 1, 0, rt.comm_unique_id())
    streams = [torch.cuda.Stream() for _ in range(3)]
    frames = [torch.zeros((spec.height, spec.width, 4), dtype=torch.uint8, device="cuda") for _ in range(5)]
    for k, f in enumerate(frames):  # no host sync in between: slot reuse is ordered by the library's events
        comm.render_strips(spec.width, spec.height, f, streams[k % 3].cuda_stream)
    comm.synchronize()
    o8, _, _ = oracle.Scene(spec).render_spec(spec, nthreads=16, want_float=False, schedule=1)
    for k, f in enumerate(frames):
        assert np.array_equal(f.cpu().numpy(), o8), f"frame {k}"
    # a new frame size re-plans the strips (the pipeline drains first)
    small = spec.with_size(333, 197)
    g = torch.zeros((small.height, small.width, 4), dtype=torch.uint8, device="cuda")
    c.set_camera(small.camera_buffer())
    comm.render_strips(small.width, small.height, g, None, 4)
    comm.synchronize()
    s8, _, _ = oracle.Scene(small).render_spec(small, nthreads=16, want_float=False, schedule=1)
    assert np.array_equal(g.cpu().numpy(), s8)
    with pytest.raises(rt.RtError):
        comm.render_strips(spec.width, spec.height, None)  # rank 0 needs the frame buffer
    comm.close()
    c.close()


def test_render_strips_moved_slots_shared_frames_and_join():
    """Slots moved between caller streams (events), two frame buffers shared by six frames on three streams (the
    assemblies into one buffer stay in call order, so each holds its LAST frame), a camera change per frame, and
    completion seen through rt_comm_stream alone (it joins the render streams, where the assemblies run)."""
    base = scenes.config("C2F").with_size(480, 272)
    c = rt.Context(0)
    scenes.upload(c, base)
    comm = rt.Comm(c, 1, 0, rt.comm_unique_id())
    streams = [torch.cuda.Stream() for _ in range(3)]
    bufs = [torch.zeros((base.height, base.width, 4), dtype=torch.uint8, device="cuda") for _ in range(2)]
    eyes = [(1.5 + 0.4 * k, 1.2 + 0.1 * k, 3.5 - 0.3 * k) for k in range(6)]
    order = [2, 0, 1, 1, 0, 2]  # call k's stream: slot k % 3 lands on another stream than its last use
    specs = []
    for k in range(6):
        sp = base.with_size(base.width, base.height)
        sp.camera = (eyes[k], (0.0, 0.5, 0.0), (0.0, 1.0, 0.0))
        specs.append(sp)
        c.set_camera(sp.camera_buffer())
        comm.render_strips(sp.width, sp.height, bufs[k % 2], streams[order[k]].cuda_stream)
    torch.cuda.ExternalStream(comm.stream).synchronize()  # no rt_comm_synchronize: the join alone
    for b, last in ((0, 4), (1, 5)):
        o8, _, _ = oracle.Scene(specs[last]).render_spec(specs[last], nthreads=16, want_float=False, schedule=1)
        assert np.array_equal(bufs[b].cpu().numpy(), o8), f"buffer {b} != frame {last}"
    comm.close()
    c.close()


@pytest.mark.parametrize("batch", [2, 3])
def test_render_strips_batched_gathers(batch):
    """rt_comm_set_batch: `batch` consecutive frames share one slot and ONE ncclGather. Seven frames with a camera
    change each (the last slot only partly filled: gathered as it is at rt_comm_synchronize), every frame into its
    own buffer, the library's own render streams; then two buffers shared by five frames on caller streams. Every
    frame equals the oracle's."""
    base = scenes.config("C2F").with_size(320, 184)
    c = rt.Context(0)
    scenes.upload(c, base)
    comm = rt.Comm(c, 1, 0, rt.comm_unique_id())
    comm.set_batch(batch)
    assert comm.batch == batch and comm.depth % batch == 0
    specs, bufs = [], []
    for k in range(7):
        sp = base.with_size(base.width, base.height)
        sp.camera = ((1.5 + 0.3 * k, 1.0 + 0.1 * k, 3.0 - 0.2 * k), (0.0, 0.5, 0.0), (0.0, 1.0, 0.0))
        specs.append(sp)
        bufs.append(torch.zeros((sp.height, sp.width, 4), dtype=torch.uint8, device="cuda"))
        c.set_camera(sp.camera_buffer())
        comm.render_strips(sp.width, sp.height, bufs[k], None)
    comm.synchronize()
    for k in range(7):
        o8, _, _ = oracle.Scene(specs[k]).render_spec(specs[k], nthreads=16, want_float=False, schedule=1)
        assert np.array_equal(bufs[k].cpu().numpy(), o8), f"frame {k}"
    streams = [torch.cuda.Stream() for _ in range(2)]
    shared = [torch.zeros((base.height, base.width, 4), dtype=torch.uint8, device="cuda") for _ in range(2)]
    for k in range(5):
        c.set_camera(specs[k].camera_buffer())
        comm.render_strips(base.width, base.height, shared[k % 2], streams[k % 2].cuda_stream)
    torch.cuda.ExternalStream(comm.stream).synchronize()
    for b, last in ((0, 4), (1, 3)):
        o8, _, _ = oracle.Scene(specs[last]).render_spec(specs[last], nthreads=16, want_float=False, schedule=1)
        assert np.array_equal(shared[b].cpu().numpy(), o8), f"shared buffer {b} != frame {last}"
    with pytest.raises(rt.RtError):
        comm.set_batch(0)
    with pytest.raises(rt.RtError):
        comm.set_batch(5)
    comm.close()
    c.close()
