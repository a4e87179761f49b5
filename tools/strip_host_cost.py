"""Host cost of one strips-mode step (bench.py's N > 1 loop) measured on ONE GPU.

For a share N (the rows rank 0 renders when a 1080p frame is tiled over N ranks) this times, per
frame: (a) the strip render alone, GPU events, back to back; (b) bench.py's step — render on one
stream, RCCL gather + rt_assemble_strips on a second, two slots, events — with a world-1 RCCL
process group (the gather moves nothing, so what is left over the render is host and launch cost);
(c) the same step replayed from a HIP graph when --graph is given and capture succeeds.
  python tools/strip_host_cost.py --shares 1,2,4,8 [--graph]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import distributed as D, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--shares", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--render-high", action="store_true", help="render stream at high priority")
    ap.add_argument("--breakdown", action="store_true", help="host cost of the step's parts")
    ap.add_argument("--graph-only", action="store_true", help="skip the eager loops (a fresh process per capture)")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    spec = scenes.config(a.config)
    ctx = rt.Context(0)
    scenes.upload(ctx, spec)
    W, H = spec.width, spec.height
    out = {}
    for n in [int(x) for x in a.shares.split(",")]:
        rows, rpr = D.rank_rows(H, n, 0), D.padded_rows(H, n)
        render = torch.cuda.Stream(dev, priority=-1 if a.render_high else 0)
        comm = torch.cuda.Stream(dev)
        local = [torch.zeros((rpr, W, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
        gathered = [torch.zeros((1, rpr, W, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
        asm_in = torch.zeros((n, rpr, W, 4), dtype=torch.uint8, device=dev)
        frame = [torch.zeros((H, W, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
        parts = [D.gather_parts(g, 1, 0) for g in gathered]
        rendered = [torch.cuda.Event() for _ in range(2)]
        freed = [torch.cuda.Event() for _ in range(2)]

        def step(k):
            s = k % 2
            render.wait_event(freed[s])
            ctx.dispatch(W, H, local[s], None, rows=rows, stream=render.cuda_stream)
            rendered[s].record(render)
            comm.wait_event(rendered[s])
            with torch.cuda.stream(comm):
                D.gather_strips(local[s], 1, 0, gathered[s], parts=parts[s])
                ctx.assemble_strips(W, H, n, D.STRIP_ROWS, asm_in, frame[s], stream=comm.cuda_stream)
            freed[s].record(comm)

        def timed(fn, frames):
            for k in range(50):
                fn(k)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(render)
            for k in range(frames):
                fn(k)
            e1.record(render)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e3 / frames, e0.elapsed_time(e1) / frames

        def step_nogather(k):
            s = k % 2
            render.wait_event(freed[s])
            ctx.dispatch(W, H, local[s], None, rows=rows, stream=render.cuda_stream)
            rendered[s].record(render)
            comm.wait_event(rendered[s])
            ctx.assemble_strips(W, H, n, D.STRIP_ROWS, asm_in, frame[s], stream=comm.cuda_stream)
            freed[s].record(comm)

        def step_cur(k):  # comm is the current stream for the whole loop: no stream context per step
            s = k % 2
            render.wait_event(freed[s])
            ctx.dispatch(W, H, local[s], None, rows=rows, stream=render.cuda_stream)
            rendered[s].record(render)
            comm.wait_event(rendered[s])
            D.gather_strips(local[s], 1, 0, gathered[s], parts=parts[s])
            ctx.assemble_strips(W, H, n, D.STRIP_ROWS, asm_in, frame[s], stream=comm.cuda_stream)
            freed[s].record(comm)

        def render_rec(k):  # render + an event record per frame, no cross-stream wait
            s = k % 2
            ctx.dispatch(W, H, local[s], None, rows=rows, stream=render.cuda_stream)
            rendered[s].record(render)

        idle = torch.cuda.Event()
        idle.record(comm)

        def render_wait(k):  # render after waiting on an event of the (idle) comm stream
            s = k % 2
            render.wait_event(idle)
            ctx.dispatch(W, H, local[s], None, rows=rows, stream=render.cuda_stream)

        def render_asm(k):  # render, then assemble on the same stream (no events)
            s = k % 2
            ctx.dispatch(W, H, local[s], None, rows=rows, stream=render.cuda_stream)
            ctx.assemble_strips(W, H, n, D.STRIP_ROWS, asm_in, frame[s], stream=render.cuda_stream)

        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        hip.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]

        def hev():
            e = ctypes.c_void_p()
            assert hip.hipEventCreateWithFlags(ctypes.byref(e), 0x2 | 0x20000000) == 0
            return e
        h_rendered, h_freed = [hev() for _ in range(2)], [hev() for _ in range(2)]
        rs, cs = ctypes.c_void_p(render.cuda_stream), ctypes.c_void_p(comm.cuda_stream)

        def step_nofence(k):  # bench's step with device-scope events (no system fence on record)
            s = k % 2
            hip.hipStreamWaitEvent(rs, h_freed[s], 0)
            ctx.dispatch(W, H, local[s], None, rows=rows, stream=render.cuda_stream)
            hip.hipEventRecord(h_rendered[s], rs)
            hip.hipStreamWaitEvent(cs, h_rendered[s], 0)
            D.gather_strips(local[s], 1, 0, gathered[s], parts=parts[s])
            ctx.assemble_strips(W, H, n, D.STRIP_ROWS, asm_in, frame[s], stream=comm.cuda_stream)
            hip.hipEventRecord(h_freed[s], cs)

        def render_rec_nofence(k):
            s = k % 2
            ctx.dispatch(W, H, local[s], None, rows=rows, stream=render.cuda_stream)
            hip.hipEventRecord(h_rendered[s], rs)

        r = {"rows": len(rows)}
        if a.breakdown:
            r["render_rec_nofence_ms"], _ = timed(render_rec_nofence, a.frames)
            with torch.cuda.stream(comm):
                r["step_nofence_ms"], _ = timed(step_nofence, a.frames)
            r["render_rec_ms"], _ = timed(render_rec, a.frames)
            r["render_wait_ms"], _ = timed(render_wait, a.frames)
            r["render_asm_ms"], _ = timed(render_asm, a.frames)
            r["nogather_wall_ms"], _ = timed(step_nogather, a.frames)
            with torch.cuda.stream(comm):
                r["curstream_wall_ms"], _ = timed(step_cur, a.frames)
            t0 = time.perf_counter()
            with torch.cuda.stream(comm):
                for k in range(a.frames):
                    D.gather_strips(local[0], 1, 0, gathered[0], parts=parts[0])
            r["gather_host_us"] = (time.perf_counter() - t0) * 1e6 / a.frames
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.frames):
                ctx.assemble_strips(W, H, n, D.STRIP_ROWS, asm_in, frame[0], stream=comm.cuda_stream)
            r["assemble_host_us"] = (time.perf_counter() - t0) * 1e6 / a.frames
            torch.cuda.synchronize()
        if a.graph_only:
            r["render_wall_ms"], r["render_gpu_ms"] = 0.0, 0.0
        else:
            r["render_wall_ms"], r["render_gpu_ms"] = timed(
                lambda k: ctx.dispatch(W, H, local[0], None, rows=rows, stream=render.cuda_stream), a.frames)
            r["step_wall_ms"], r["step_render_stream_ms"] = timed(step, a.frames)
        t0 = time.perf_counter()
        for k in range(a.frames):
            ctx.dispatch(W, H, local[0], None, rows=rows, stream=render.cuda_stream)
        r["dispatch_host_us"] = (time.perf_counter() - t0) * 1e6 / a.frames
        torch.cuda.synchronize()
        if a.graph:
            try:
                g = torch.cuda.CUDAGraph()
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=render):
                    for k in range(8):
                        step(k)
                    render.wait_stream(comm)  # join the last gathers into the capture
                torch.cuda.synchronize()
                reps = max(1, a.frames // 8)
                r["graph_wall_ms"], _ = timed(lambda k: g.replay(), reps)
                r["graph_wall_ms"] /= 8
            except Exception as e:  # noqa: BLE001
                r["graph_error"] = repr(e)[:300]
        out[f"N{n}"] = r
        print(n, json.dumps(r), flush=True)
    ctx.close()
    dist.destroy_process_group()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
