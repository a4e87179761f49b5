"""N>1 path on CPU: world_size 2 (and 3) gloo process groups run the same partition -> render ->
gather -> un-interleave sequence as bench.py's RCCL path. Each rank renders its strips with the
CPU oracle (the only renderer available without a GPU); the assembled frame must equal a
single-process full-frame render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, name, size, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from realtimeraytracing_gradproject_amd import distributed as D, scenes
        spec = scenes.config(name).with_size(*size)
        rows = D.rank_rows(spec.height, world, rank)
        pad = D.padded_rows(spec.height, world)
        o8, _, _ = oracle.Scene(spec).render_spec(spec, rows=rows, nthreads=2, want_float=False)
        local = torch.zeros((pad, spec.width, 4), dtype=torch.uint8)
        local[: len(rows)] = torch.from_numpy(o8)
        gathered = torch.zeros((world, pad, spec.width, 4), dtype=torch.uint8) if rank == 0 else None
        D.gather_strips(local, world, rank, gathered)
        # ranks agree on the ray count of the frame (all_reduce, as bench.py does)
        n = torch.tensor([float(len(rows))])
        dist.all_reduce(n)
        if rank == 0:
            q.put((D.assemble_host(gathered.numpy(), spec.height, world), float(n.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name,size", [(2, "C2F", (64, 36)), (3, "C4", (40, 29))])
def test_gloo_strip_gather_assemble(world, name, size):
    import sys
    sys.path.insert(0, ROOT)
    import oracle
    from realtimeraytracing_gradproject_amd import scenes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, name, size, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame, nrows = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    spec = scenes.config(name).with_size(*size)
    full8, _, _ = oracle.Scene(spec).render_spec(spec, nthreads=2, want_float=False)
    assert nrows == spec.height
    assert np.array_equal(frame, full8)


def test_assemble_host_inverse_of_partition():
    from realtimeraytracing_gradproject_amd import distributed as D
    H, W = 77, 5
    full = np.arange(H * W * 4, dtype=np.uint32).reshape(H, W, 4)
    for world in (1, 2, 4, 8):
        pad = D.padded_rows(H, world)
        g = np.zeros((world, pad, W, 4), np.uint32)
        for r in range(world):
            rows = D.rank_rows(H, world, r)
            g[r, : len(rows)] = full[rows]
        assert np.array_equal(D.assemble_host(g, H, world), full)


def frames_worker(rank, world, port, name, size, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from realtimeraytracing_gradproject_amd import scenes
        spec = scenes.config(name).with_size(*size)
        o8, _, st = oracle.Scene(spec).render_spec(spec, nthreads=1, want_float=False)
        # bench.py's default N>1 mode: each rank renders a whole frame, no data-path collective;
        # only the ray counts (sum) and the timed wall clock (max) are reduced
        counts = torch.tensor([float(st[0] + st[1])], dtype=torch.float64)
        dist.all_reduce(counts)
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, o8, float(st[0] + st[1]), float(counts.item()), float(t.item())))
    finally:
        dist.destroy_process_group()


def test_gloo_frames_mode_weak():
    """Weak-scaling frames mode: N ranks, N identical frames, rays per step = N x one frame."""
    import sys
    sys.path.insert(0, ROOT)
    world, name, size = 2, "C2F", (48, 27)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=frames_worker, args=(r, world, port, name, size, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert np.array_equal(res[0][1], res[1][1])
    for _, _, local, total, tmax in res:
        assert total == world * local
        assert tmax == float(world)


@pytest.mark.parametrize("world", [2, 8])
def test_bench_spawn_path_gloo(tmp_path, world):
    """bench.py's own N>1 path end to end on CPU: `bench.py --gpus N` (no WORLD_SIZE) re-launches
    itself under torch.distributed.run, the ranks tile one frame into strips, gather and assemble
    it (pipelined, two slots), all-reduce the counters and max-reduce the clock; rank 0 prints the
    JSON line. The test backend swaps the HIP renderer for the oracle (gloo, CPU tensors)."""
    import json
    import subprocess
    import sys
    sys.path.insert(0, ROOT)
    import oracle
    from realtimeraytracing_gradproject_amd import scenes
    img = tmp_path / "frame.npy"
    env = dict(os.environ, RT_BENCH_TEST_BACKEND="tests.bench_cpu_backend:CpuBackend",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    # 64 x 44: 6 strips of 8 rows, so at N = 8 two ranks render nothing (ragged partition)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--config", "C2F", "--size", "64x44",
           # a clock settle on: ranks with unequal strip shares must still agree on its step count
           "--steps", "3", "--warmup", "1", "--settle-ms", "30", "--extra", "C4", "--no-cpu-baseline",
           "--save-image", str(img)]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["scaling"] == "strong"
    assert out["config"]["rccl_world_size"] == world
    assert out["config"]["parallelism"].startswith(f"strips{world}+gather")
    spec = scenes.config("C2F").with_size(64, 44)
    o8, _, st = oracle.Scene(spec).render_spec(spec, nthreads=2, want_float=False)
    assert out["config"]["rays_per_step"] == int(st[0] + st[1])  # one frame's rays over both ranks
    assert np.array_equal(np.load(img), o8)  # assembled from both ranks' strips, bit for bit
    assert [e["config"] for e in out["extra"]] == ["C4"] and out["extra"][0]["n_gpus"] == world
    assert out["roofline"]["frac"] <= 1.0


def test_bench_native_comm_failure_falls_back_together(tmp_path):
    """bench.py asked for the native RCCL loop, but rt_comm_init returns an error on one rank (here simulated on rank
    1 alone, the other rank's init returning normally): the ranks agree (all-reduce MIN) and all of them run the
    torch.distributed strips loop rather than issuing gathers on a communicator that one rank lacks; the assembled
    frame is still the oracle's. (A rank that never returns from ncclCommInitRank cannot be recovered this way.)"""
    import json
    import subprocess
    import sys
    sys.path.insert(0, ROOT)
    import oracle
    from realtimeraytracing_gradproject_amd import scenes
    img = tmp_path / "frame.npy"
    env = dict(os.environ, RT_BENCH_TEST_BACKEND="tests.bench_cpu_backend:CpuBackendCommFails", RCCL_FAIL_RANK="1",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C2F", "--size", "64x44",
           "--steps", "3", "--warmup", "1", "--settle-ms", "10", "--resettle-ms", "0", "--extra=", "--no-cpu-baseline",
           "--save-image", str(img)]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "simulated RCCL failure" in p.stderr
    assert "comm aborted on rank 0" in p.stderr  # rank 0's communicator came up: aborted, no collective on it
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["config"]["strips_loop"] == "torch.distributed gather"
    spec = scenes.config("C2F").with_size(64, 44)
    o8, _, _ = oracle.Scene(spec).render_spec(spec, nthreads=2, want_float=False)
    assert np.array_equal(np.load(img), o8)


def test_bench_native_loop_error_aborts_communicator(tmp_path):
    """An error inside bench.py's native strips loop (the render call raises on its 3rd call, a partly filled batch
    of 4 pending): the communicator is aborted (rt_comm_abort: no draining gather the other ranks might never match,
    VERDICT r4 #7), not closed, and the error propagates (non-zero exit)."""
    import subprocess
    import sys
    env = dict(os.environ, RT_BENCH_TEST_BACKEND="tests.bench_cpu_backend:CpuBackendStepFails", STEP_FAIL_AT="3",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--mode", "strips", "--config", "C2F", "--size", "64x44",
           "--steps", "3", "--warmup", "4", "--settle-ms", "0", "--resettle-ms", "0", "--extra=", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert p.returncode != 0
    assert "simulated render failure" in p.stderr
    assert "comm aborted" in p.stderr and "comm closed" not in p.stderr, p.stderr[-3000:]


def test_bench_native_loop_phases_gloo(tmp_path):
    """the N > 1 line names its own binding cost. bench.py's native strips loop at world 2 (a stand-in
    communicator over gloo that renders, gathers and assembles, timing each phase as rt_comm_phase_stats reports
    them): config.phases carries the render share (with its max / min over the ranks), the gather, the assembly, the
    host issue per frame, the bytes into rank 0 and their rate, and the period; the assembled frame is the oracle's."""
    import json
    import subprocess
    import sys
    sys.path.insert(0, ROOT)
    import oracle
    from realtimeraytracing_gradproject_amd import scenes
    img = tmp_path / "frame.npy"
    env = dict(os.environ, RT_BENCH_TEST_BACKEND="tests.bench_cpu_backend:CpuBackendNative",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C2F", "--size", "64x44",
           "--steps", "3", "--warmup", "1", "--settle-ms", "0", "--resettle-ms", "0", "--extra=", "--no-cpu-baseline",
           "--phase-frames", "4", "--latency-frames", "2", "--save-image", str(img)]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    ph = out["config"]["phases"]
    assert ph["frames"] == 4 and ph["world"] == 2 and ph["rank"] == 0
    assert ph["render_share_ms_max"] >= ph["render_share_ms"] >= ph["render_share_ms_min"] > 0
    assert ph["gather_ms"] > 0 and ph["assembly_ms"] > 0 and ph["host_issue_us"] > 0
    # rank 1's padded strip block (3 strips of 8 rows), one block per call of 4 frames (the stand-in gathers once)
    assert ph["bytes_into_rank0_per_frame"] == 24 * 64 * 4 // 4
    assert ph["ingress_GBps_over_gather"] > 0 and ph["period_ms"] > 0
    assert 0.5 <= ph["phase_sum_over_period"] <= 1.5  # one thread runs the phases back to back: they are the period
    spec = scenes.config("C2F").with_size(64, 44)
    o8, _, _ = oracle.Scene(spec).render_spec(spec, nthreads=2, want_float=False)
    assert np.array_equal(np.load(img), o8)
