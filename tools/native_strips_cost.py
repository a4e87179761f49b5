"""Host issue cost of one tiled-frame step: the C-ABI's rt_render_strips (render -> ncclGather ->
assembly issued from C++) against bench.py's former Python step (torch.distributed gather + rt_event_* +
rt_assemble_strips), both over a world-1 RCCL group on ONE GPU (the gather moves nothing: what is measured is the
host and launch cost of a step). Per loop: the host time to ISSUE `frames` steps (no synchronisation inside the
loop; the GPU is kept busy so issue is not throttled by an empty queue; for the native loop this is the caller's
thread, the library's issue thread runs the gather half beside it), and the wall time per frame once everything
has drained, with 1 and 3 render streams (frames in flight). RT_COMM_TIMING=1 prints both threads' breakdown.

  python tools/native_strips_cost.py --config C2 --frames 200 > gpurun_out/native_strips_cost.json
"""
import argparse
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
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--size", default="", help="WxH: e.g. 1920x136, the rows one of 8 ranks renders, so the GPU "
                                                "time per frame is small enough that the host issue shows")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29534")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    spec = scenes.config(a.config)
    if a.size:
        spec = spec.with_size(*(int(v) for v in a.size.lower().split("x")))
    W, H = spec.width, spec.height
    ctx = rt.Context(0)
    scenes.upload(ctx, spec)
    comm = rt.Comm(ctx, 1, 0, rt.comm_unique_id())
    nslot = 4
    frames = [torch.zeros((H, W, 4), dtype=torch.uint8, device=dev) for _ in range(max(nslot, comm.depth))]
    streams = [torch.cuda.Stream(dev) for _ in range(3)]

    # --- the former Python step (bench.py before rt_render_strips) ---------------------------------
    rows, rpr = D.rank_rows(H, 1, 0), D.padded_rows(H, 1)
    cstream = torch.cuda.Stream(dev)
    local = [torch.zeros((rpr, W, 4), dtype=torch.uint8, device=dev) for _ in range(nslot)]
    gathered = [torch.zeros((1, rpr, W, 4), dtype=torch.uint8, device=dev) for _ in range(nslot)]
    parts = [D.gather_parts(g, 1, 0) for g in gathered]
    rendered = [rt.PipelineEvent() for _ in range(nslot)]
    freed = [rt.PipelineEvent() for _ in range(nslot)]
    used = [False] * nslot

    def py_step(k, nstream):
        s = k % nslot
        rs = streams[s % nstream]
        if used[s]:
            freed[s].wait_on(rs.cuda_stream)
        ctx.dispatch(W, H, local[s], None, rows=rows, stream=rs.cuda_stream)
        rendered[s].record(rs.cuda_stream)
        rendered[s].wait_on(cstream.cuda_stream)
        D.gather_strips(local[s], 1, 0, gathered[s], parts=parts[s])
        ctx.assemble_strips(W, H, 1, D.STRIP_ROWS, gathered[s], frames[s], stream=cstream.cuda_stream)
        freed[s].record(cstream.cuda_stream)
        used[s] = True

    depth = comm.depth
    ncall = [0]  # the library's slot is its call count mod depth: stream i serves slot i (no slot moves streams)

    def native_step(k, nstream):
        si = ncall[0] % depth
        ncall[0] += 1
        comm.render_strips(W, H, frames[si], streams[si % nstream].cuda_stream)

    def sync():
        comm.synchronize()  # the library's issue thread has enqueued every handed-over gather
        torch.cuda.synchronize()

    def measure(fn, nstream):
        best_issue, best_frame = float("inf"), float("inf")
        for _ in range(a.rounds):
            for k in range(20):
                fn(k, nstream)
            sync()
            t0 = time.perf_counter()
            for k in range(a.frames):
                fn(k, nstream)
            t1 = time.perf_counter()
            sync()
            t2 = time.perf_counter()
            best_issue = min(best_issue, (t1 - t0) * 1e6 / a.frames)
            best_frame = min(best_frame, (t2 - t0) * 1e3 / a.frames)
        return {"host_issue_us_per_step": round(best_issue, 2), "ms_per_frame": round(best_frame, 4)}

    out = {"config": a.config, "size": f"{W}x{H}", "frames": a.frames, "world": 1, "pipeline_depth": comm.depth,
           "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
    with torch.cuda.stream(cstream):
        out["python_step_1stream"] = measure(py_step, 1)
        out["python_step_3streams"] = measure(py_step, 3)
    out["native_step_1stream"] = measure(native_step, 1)
    out["native_step_3streams"] = measure(native_step, 3)

    def native_own(k, nstream):  # render_stream NULL: the communicator's own three render streams
        si = ncall[0] % depth
        ncall[0] += 1
        comm.render_strips(W, H, frames[si], None)
    out["native_step_library_streams"] = measure(native_own, 3)
    for b in (2, 4):  # rt_comm_set_batch: b frames per ncclGather (the gather half paid once per b frames)
        comm.set_batch(b)
        depth = comm.depth
        while len(frames) < depth:
            frames.append(torch.zeros((H, W, 4), dtype=torch.uint8, device=dev))
        ncall[0] = 0
        out[f"native_step_library_streams_batch{b}"] = measure(native_own, 3)
    comm.set_batch(1)
    depth = comm.depth
    # host cost of the call alone while the GPU is idle-free: the render itself issued alone
    t0 = time.perf_counter()
    for k in range(a.frames):
        ctx.dispatch(W, H, frames[k % nslot], None, stream=streams[0].cuda_stream)
    out["dispatch_alone_host_us"] = round((time.perf_counter() - t0) * 1e6 / a.frames, 2)
    torch.cuda.synchronize()
    comm.close()
    ctx.close()
    dist.destroy_process_group()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
