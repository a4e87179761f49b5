"""The CPU oracle itself: LBVH invariants, BVH == brute force, shading known answers, the
independent numpy restatement, and the committed golden frames (tests/golden/frames_small.npz)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import realtimeraytracing_gradproject_amd as rt
from realtimeraytracing_gradproject_amd import scenes
import oracle
from oracle import np_reference

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "frames_small.npz"))
SIZES = {"REF": (96, 54), "C1": (64, 64), "C2": (96, 54), "C2F": (96, 54), "C3": (96, 54), "C4": (96, 54),
         "C5": (48, 27), "REFL": (96, 54), "REFLO": (96, 54), "DEGEN": (96, 54)}


EMPTY = np.int32(-2**31 + 1)


def unpack4(nodes):
    """128-B 4-wide nodes -> lo (n,4,3), hi (n,4,3), child (n,4), count (n,)."""
    f = nodes.view(np.float32)
    lo = np.stack([f[:, 0:4], f[:, 8:12], f[:, 16:20]], -1)
    hi = np.stack([f[:, 4:8], f[:, 12:16], f[:, 20:24]], -1)
    return lo, hi, nodes[:, 24:28].view(np.int32), nodes[:, 28]


@pytest.mark.parametrize("model", ["teapot", "rabbit"])
def test_lbvh_invariants(model):
    v, i = scenes.load_model(model)
    o = oracle.Scene()
    b = o.add_blas(v, i)
    nodes, tris = o.export_blas(b)
    lo, hi, ch, count = unpack4(nodes)
    n = tris.shape[0]
    valid = ch != EMPTY
    assert (valid.sum(1) == count).all() and (count >= 2).all() and (count <= 4).all()
    # every primitive exactly once in leaf order; every leaf slot referenced exactly once
    assert np.array_equal(np.sort(tris[:, 3]), np.arange(n))
    leaves = ~ch[valid & (ch < 0)]
    assert np.array_equal(np.sort(leaves), np.arange(n))
    # every node but the root has exactly one parent, and BFS order puts children after parents
    internal = ch[valid & (ch >= 0)]
    assert np.array_equal(np.sort(internal), np.arange(1, len(nodes)))
    parents = np.repeat(np.arange(len(nodes))[:, None], 4, 1)[valid & (ch >= 0)]
    assert (internal > parents).all()
    # a child box is exactly the union of that child's own child boxes (refit exactness)
    for k in range(len(nodes)):
        for j in range(4):
            c = ch[k, j]
            if c >= 0:
                m = ch[c] != EMPTY
                assert np.array_equal(lo[k, j], lo[c][m].min(0)) and np.array_equal(hi[k, j], hi[c][m].max(0))
    # leaf boxes contain their triangle
    tf = tris.view(np.float32)
    v0, e1, e2 = tf[:, 0:3], tf[:, 4:7], tf[:, 8:11]
    pts = np.stack([v0, v0 + e1, v0 + e2], 1)
    for k, j in zip(*np.nonzero(valid & (ch < 0))):
        p = pts[~ch[k, j]]
        assert (p >= lo[k, j] - 1e-6).all() and (p <= hi[k, j] + 1e-6).all()


@pytest.mark.parametrize("model", ["teapot", "rabbit"])
def test_node_meta_for_packet_stack(model):
    """first_inner / inner_mask / entry_base (the packet walk's one-entry-per-node stack):
    internal children have consecutive refs in slot order, starting at first_inner."""
    v, i = scenes.load_model(model)
    o = oracle.Scene()
    nodes, _ = o.export_blas(o.add_blas(v, i))
    u = nodes.view(np.uint32).reshape(-1, 32)
    ch = u[:, 24:28].view(np.int32)
    for k in range(len(u)):
        inner = [j for j in range(4) if ch[k, j] >= 0]
        mask = sum(1 << j for j in inner)
        assert u[k, 30] == mask
        if inner:
            refs = [ch[k, j] for j in inner]
            assert refs == list(range(refs[0], refs[0] + len(refs)))
            assert u[k, 29] == refs[0]
        assert u[k, 31] == ((int(u[k, 29]) << 8) | (mask << 4))


@pytest.mark.parametrize("model", ["teapot", "rabbit"])
def test_slots_in_ascending_area(model):
    """BLAS nodes hold their internal children first, then their triangles, each group by ascending
    half area (stable): the nearest-first walk breaks key ties (rays starting inside several boxes)
    and any-hit walks go lowest slot first, both then enter the tighter box first; triangles are
    tested in place, so only the internal children's order matters, and internal child k is
    first_inner + k."""
    v, i = scenes.load_model(model)
    o = oracle.Scene()
    nodes, _ = o.export_blas(o.add_blas(v, i))
    lo, hi, ch, count = unpack4(nodes)
    d = (hi - lo).astype(np.float32)
    area = (d[..., 0] * d[..., 1] + d[..., 1] * d[..., 2]) + d[..., 2] * d[..., 0]
    first_inner = nodes.view(np.int32)[:, 29]
    for k in range(len(nodes)):
        inner = ch[k, :count[k]] >= 0
        ni = int(inner.sum())
        assert inner[:ni].all() and not inner[ni:].any()
        for grp in (area[k, :ni], area[k, ni:count[k]]):
            assert (grp[1:] >= grp[:-1]).all()
        assert np.array_equal(ch[k, :ni], first_inner[k] + np.arange(ni))


def _wide_area(model: str, greedy: bool) -> float:
    """Sum of the wide nodes' half areas (the collapse's SAH cost) from a fresh process: the oracle
    reads ORACLE_GREEDY_COLLAPSE once."""
    code = (
        "import sys, numpy as np; sys.path.insert(0, %r)\n"
        "import oracle\nfrom realtimeraytracing_gradproject_amd import scenes\n"
        "v, i = scenes.load_model(%r); o = oracle.Scene(); n, _ = o.export_blas(o.add_blas(v, i))\n"
        "f = n.view(np.float32).reshape(-1, 32).astype(np.float64); c = n.view(np.int32).reshape(-1, 32)[:, 24:28]\n"
        "m = c != -2147483647\n"
        "lo = np.stack([np.where(m, f[:, 0:4], np.inf).min(1), np.where(m, f[:, 8:12], np.inf).min(1),"
        " np.where(m, f[:, 16:20], np.inf).min(1)], 1)\n"
        "hi = np.stack([np.where(m, f[:, 4:8], -np.inf).max(1), np.where(m, f[:, 12:16], -np.inf).max(1),"
        " np.where(m, f[:, 20:24], -np.inf).max(1)], 1)\n"
        "d = hi - lo; print(float((d[:, 0] * d[:, 1] + d[:, 1] * d[:, 2] + d[:, 2] * d[:, 0]).sum()), len(n))\n"
    ) % (ROOT, model)
    env = dict(os.environ)
    env.pop("ORACLE_GREEDY_COLLAPSE", None)
    if greedy:
        env["ORACLE_GREEDY_COLLAPSE"] = "1"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    area, nn = out.stdout.split()
    return float(area), int(nn)


@pytest.mark.parametrize("model", ["teapot", "rabbit"])
def test_sah_collapse_beats_greedy(model):
    """The DP collapse (the product's default, mirrored here) minimises the summed wide-node area:
    never worse than the greedy largest-area opening it replaced, and fewer nodes on these meshes."""
    dp, n_dp = _wide_area(model, greedy=False)
    gr, n_gr = _wide_area(model, greedy=True)
    assert dp <= gr * (1 + 1e-6)
    assert n_dp < n_gr


@pytest.mark.parametrize("name", ["REF", "C1", "C2F", "C3", "C4", "DEGEN"])
def test_bvh_image_equals_bruteforce(name):
    spec = scenes.config(name).with_size(48, 27)
    o = oracle.Scene(spec)
    a8, a32, _ = o.render_spec(spec, nthreads=8)
    b8, b32, _ = o.render_spec(spec, nthreads=8, brute_force=True)
    assert np.array_equal(a32, b32) and np.array_equal(a8, b8)


@pytest.mark.parametrize("name,size", [("C2", (480, 270)), ("C2F", (480, 270)), ("C3", (320, 180)),
                                       ("C4", (320, 180)), ("REF", (320, 180)), ("DEGEN", (256, 144))])
def test_packet_schedule_image_equals_per_ray(name, size):
    """The packet emulation (the device's default schedule) renders the per-ray schedule's image (which equals brute
    force above) on larger frames and a seeded camera sweep around each scene: the slab test's conservative widening
    holds on every ray. (This test refuted the far-plane prescale of VERDICT r3 #5: with the widening folded into
    pre-scaled far-plane terms, three DEGEN shadow rays at 256 x 144 lost their occluder)"""
    base = scenes.config(name) if name != "DEGEN" else scenes.degenerate_scene()
    spec = base.with_size(*size)
    o = oracle.Scene(spec)
    a8, a32, _ = o.render_spec(spec, nthreads=8, want_float=True, schedule=0)
    b8, b32, _ = o.render_spec(spec, nthreads=8, want_float=True, schedule=1)
    assert np.array_equal(a32, b32) and np.array_equal(a8, b8), name
    rng = np.random.default_rng(0x5EED + len(name))
    for _ in range(3):
        eye = tuple(float(x) for x in rng.uniform(-1, 1, 3) * [12, 6, 12] + [0, 7, 0])
        sp = base.with_size(160, 90)
        sp.camera = (eye, tuple(float(x) for x in rng.uniform(-1, 1, 3) * [2, 1, 2]), (0.0, 1.0, 0.0))
        a8, _, _ = o.render_spec(sp, nthreads=8, want_float=False, schedule=0)
        b8, _, _ = o.render_spec(sp, nthreads=8, want_float=False, schedule=1)
        assert np.array_equal(a8, b8), (name, eye)


def random_rays(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.normal(size=(n, 3))
    o = o / np.linalg.norm(o, axis=1, keepdims=True) * 12 + [0, 1, 0]
    d = rng.uniform(-6, 6, size=(n, 3)) + [0, 1, 0] - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros((n, 8), np.float32)
    r[:, :3], r[:, 4:7], r[:, 7] = o, d, 1e5
    return r


@pytest.mark.parametrize("any_hit", [False, True])
def test_trace_rays_bvh_equals_bruteforce(any_hit):
    o = oracle.Scene(scenes.config("REF"))
    rays = random_rays(3000, 7)
    h1, uv1, _ = o.trace_rays(rays, any_hit=any_hit)
    h2, uv2, _ = o.trace_rays(rays, any_hit=any_hit, brute_force=True)
    if any_hit:
        assert np.array_equal(h1[:, 3], h2[:, 3])
    else:
        assert np.array_equal(h1, h2) and np.array_equal(uv1, uv2)
    assert h1[:, 3].sum() > 300


@pytest.mark.parametrize("any_hit,cull", [(False, None), (True, None), (False, "back"), (False, "front")])
def test_trace_rays_degenerate_and_transformed(any_hit, cull):
    """Degenerate triangles under rotated / scaled / mirrored instances: BVH == brute force."""
    o = oracle.Scene(scenes.config("DEGEN"))
    rays = random_rays(3000, 11)
    kw = dict(any_hit=any_hit, cull_back=cull == "back", cull_front=cull == "front")
    h1, uv1, _ = o.trace_rays(rays, **kw)
    h2, uv2, _ = o.trace_rays(rays, brute_force=True, **kw)
    if any_hit:
        assert np.array_equal(h1[:, 3], h2[:, 3])
    else:
        assert np.array_equal(h1, h2) and np.array_equal(uv1, uv2)
    assert h1[:, 3].sum() > 300


def test_tie_break_duplicate_instances():
    """Instances 1 and 2 of the reference scene coincide (D3D12HelloTriangle.cpp:785-786): the
    lower instance index wins."""
    o = oracle.Scene(scenes.config("REF"))
    r = np.zeros((1, 8), np.float32)
    r[0, :3] = (-5.0, 10.0, 5.0)
    r[0, 4:7] = (0.0, -1.0, 0.0)
    r[0, 7] = 1e5
    h, _, _ = o.trace_rays(r)
    assert h[0, 3] == 1 and h[0, 1] == 1


@pytest.mark.parametrize("name", list(SIZES))
def test_oracle_matches_golden_frames(name):
    spec = scenes.config(name).with_size(*SIZES[name])
    sc = oracle.Scene(spec)
    for sched, key in ((0, "stats"), (1, "stats_lane")):
        o8, o32, st = sc.render_spec(spec, nthreads=8, schedule=sched)
        assert np.array_equal(o8, GOLD[f"{name}_rgba8"])
        assert np.array_equal(o32.view(np.uint32), GOLD[f"{name}_rgba32f"].view(np.uint32))
        assert np.array_equal(st, GOLD[f"{name}_{key}"])


@pytest.mark.parametrize("name", ["REF", "C1", "C2F", "C3", "DEGEN", "REFLO"])
def test_oracle_vs_independent_numpy(name):
    spec = scenes.config(name).with_size(40, 24)
    img, _ = np_reference.Scene(spec).render(spec.camera_buffer())
    _, o32, _ = oracle.Scene(spec).render_spec(spec, nthreads=8)
    assert np.abs(img - o32[..., :3]).max() < 1e-4


# ------------------------------------------------------------------------------------------
# known-answer shading (Hit.hlsl / Miss.hlsl formulas evaluated by hand in float64)
# ------------------------------------------------------------------------------------------

def test_miss_gradient_kat():
    spec = scenes.config("C2").with_size(8, 10)
    spec.camera = ((0, 5, 0), (0, 50, 0.001), (0, 1, 0))  # looks straight up: every ray misses
    _, o32, st = oracle.Scene(spec).render_spec(spec)
    for y in range(10):
        assert np.allclose(o32[y, :, :3], [0.0, 0.2, 0.7 - 0.3 * (y / 10)], atol=1e-7)
    assert st[1] == 0


def test_plane_lambert_and_shadow_kat():
    spec = scenes.config("REF").with_size(1, 1)
    spec.instances = [spec.instances[-1]]  # plane only
    spec.camera = ((3.0, 2.0, 3.0), (3.0, -1.0, 3.0001), (0, 1, 0))  # straight down at (3,-1,3)
    _, o32, st = oracle.Scene(spec).render_spec(spec)
    P = np.array([3.0, -1.0, 3.0])
    L = np.array([0, 10, 0]) - P
    expect = (L / np.linalg.norm(L))[1]  # n = +Y, unshadowed
    assert abs(o32[0, 0, 0] - expect) < 1e-5 and st[1] == 1  # one shadow ray (Hit.hlsl:229)
    # same pixel with a blocker above: factor 0.3
    spec2 = scenes.config("REF").with_size(1, 1)
    spec2.camera = spec.camera
    spec2.instances = [spec2.instances[0], spec2.instances[-1]]
    spec2.instances[0] = (0, scenes.translation(0.0, 3.0, 0.0), 0, 0)
    spec2.camera = ((1.0, 0.0, 0.5), (1.0, -1.0, 0.5001), (0, 1, 0))
    _, o32b, _ = oracle.Scene(spec2).render_spec(spec2)
    P2 = np.array([1.0, -1.0, 0.5])
    L2 = np.array([0, 10, 0]) - P2
    assert abs(o32b[0, 0, 0] - 0.3 * (L2 / np.linalg.norm(L2))[1]) < 1e-5


def pbr64(n, cam, P, lights, mat):
    return np_reference.Scene._pbr(np.asarray([n], float), np.asarray([cam], float), np.asarray([P], float),
                                   [(np.array(c, float), np.array(p, float), i) for c, p, i in lights],
                                   np.asarray(mat, float))[0]


@pytest.mark.parametrize("seed", range(5))
def test_pbr_and_direct_kat(seed):
    rng = np.random.default_rng(seed)
    n = rng.normal(size=3)
    n /= np.linalg.norm(n)
    P = rng.uniform(-2, 2, size=3)
    cam = rng.uniform(-8, 8, size=3)
    mat = (1.0, 1.0, 1.0, rng.uniform(0.1, 1.0), rng.uniform(0, 1), 0.0)
    got = oracle.pbr(n, cam, P, scenes.REFERENCE_LIGHTS, mat)
    assert np.allclose(got, pbr64(n, cam, P, scenes.REFERENCE_LIGHTS, mat), atol=2e-6)
    d = oracle.direct(n, P, scenes.REFERENCE_LIGHTS, mat[:3])
    exp = sum(np.maximum(0, np.dot(n, -(np.array(p) - P) / np.linalg.norm(np.array(p) - P)) * i)
              for _, p, i in scenes.REFERENCE_LIGHTS)
    assert np.allclose(d, exp, atol=1e-6)


def test_deterministic_pow_accuracy():
    xs = np.concatenate([np.linspace(1e-6, 1, 2000), [0.5, 0.25, 1.0, 1e-20, 0.0]])
    for x in xs:
        got = oracle.pow_(float(x), 1.0 / 2.2)
        exp = float(np.float64(np.float32(x)) ** np.float64(np.float32(1 / 2.2))) if x > 1e-30 else 0.0
        assert abs(got - exp) <= 1e-6 * max(exp, 1e-3), (x, got, exp)


# ------------------------------------------------------------------------------------------
# reflection rays: back-face culling convention and the reflection chain
# ------------------------------------------------------------------------------------------

def _one_triangle_scene(xform):
    """One triangle v0=(0,0,1), v1=(0,1,1), v2=(1,0,1): seen from the origin looking +z its
    vertices run clockwise (x right, y up), i.e. it is FRONT-facing for DXR's default."""
    v = np.array([[0, 0, 1, 0, 0, -1], [0, 1, 1, 0, 0, -1], [1, 0, 1, 0, 0, -1]], np.float32)
    o = oracle.Scene()
    o.add_blas(v, None)
    o.set_instances([(0, xform, 0, rt.RT_HITGROUP_MODEL)])
    return o


def _rays(o, d):
    r = np.zeros((1, 8), np.float32)
    r[0, :3] = o
    r[0, 4:7] = d
    r[0, 7] = 100.0
    return r


def test_backface_cull_kat():
    """RAY_FLAG_CULL_BACK_FACING_TRIANGLES: clockwise-from-origin = front (DXR default); a mirroring
    instance transform (negative determinant) swaps the sides."""
    front = _rays((0.2, 0.2, 0.0), (0, 0, 1))   # sees v0, v1, v2 clockwise
    back = _rays((0.2, 0.2, 2.0), (0, 0, -1))   # sees them counter-clockwise
    o = _one_triangle_scene(scenes.IDENTITY)
    for r, expect in ((front, 1), (back, 0)):
        h, _, _ = o.trace_rays(r, cull_back=True)
        assert h[0, 3] == expect
        h, _, _ = o.trace_rays(r)  # no culling: both sides hit
        assert h[0, 3] == 1
    mirror = np.array([-1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0], np.float32)
    o = _one_triangle_scene(mirror)
    front_m = _rays((-0.2, 0.2, 0.0), (0, 0, 1))
    back_m = _rays((-0.2, 0.2, 2.0), (0, 0, -1))
    assert o.trace_rays(front_m, cull_back=True)[0][0, 3] == 0
    assert o.trace_rays(back_m, cull_back=True)[0][0, 3] == 1


@pytest.mark.parametrize("name", ["REFL", "REFLO"])
def test_reflection_chain_schedules_agree(name):
    spec = scenes.config(name).with_size(80, 45)
    sc = oracle.Scene(spec)
    a8, a32, sa = sc.render_spec(spec, nthreads=8, schedule=0)
    b8, b32, sb = sc.render_spec(spec, nthreads=8, schedule=1)
    c8, c32, _ = sc.render_spec(spec, nthreads=8, brute_force=True)
    assert np.array_equal(a32.view(np.uint32), b32.view(np.uint32))
    assert np.array_equal(a32.view(np.uint32), c32.view(np.uint32))
    assert sa[8] == sb[8] > 0  # reflection rays, same count either way
    # reflectivity 0 renders the reference image exactly (no reflection ray at all)
    ref = scenes.config("REF").with_size(80, 45)
    r8, r32, rs = oracle.Scene(ref).render_spec(ref, nthreads=8)
    if name == "REFL":
        assert rs[8] == 0 and not np.array_equal(a32, r32)


def test_reflection_chain_kat():
    """One mirror bounce by hand: camera above the plane looking down at a reflective model
    instance (InstanceID 0) whose reflection ray misses: c = (1 - r) s + r miss."""
    spec = scenes.config("REFLO").with_size(1, 1)
    spec.instances = [spec.instances[0]]  # teapot at the origin only
    spec.camera = ((0.0, 10.0, 0.001), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0))  # straight down onto the lid
    sc = oracle.Scene(spec)
    _, o32, st = sc.render_spec(spec)
    r = spec.material[5]
    # no-reflection surface colour of the same pixel and the miss colour of row 0
    plain = scenes.config("REFLO").with_size(1, 1)
    plain.instances, plain.camera = spec.instances, spec.camera
    plain.material = spec.material[:5] + (0.0,)
    _, s32, _ = oracle.Scene(plain).render_spec(plain)
    miss = np.array([0.0, 0.2, 0.7])
    assert st[8] == 1
    expect = (1.0 - r) * s32[0, 0, :3].astype(np.float64) + r * miss
    assert np.abs(o32[0, 0, :3] - expect).max() < 1e-6


@pytest.mark.parametrize("name,size", [("C2", (192, 108)), ("C4", (160, 90)), ("REFL", (96, 54)), ("DEGEN", (160, 90)),
                                       ("C5", (64, 36))])
def test_cpu_baseline_build_renders_the_checker_frames(name, size):
    """oracle/libbaseline.so (-O3, counters compiled out, plain-compare slab min/max) is the
    bench's CPU baseline; it must render exactly the checker's frames (per-ray schedule, as the bench times it)."""
    spec = scenes.config(name).with_size(*size)
    base = oracle.baseline_lib()
    assert b"-O3" in base.oracle_build_info() and b"ORACLE_NO_COUNTERS" in base.oracle_build_info()
    c8, c32, cst = oracle.Scene(spec).render_spec(spec, nthreads=4, schedule=1)
    b8, b32, bst = oracle.Scene(spec, library=base).render_spec(spec, nthreads=4, schedule=1)
    assert np.array_equal(c8, b8) and np.array_equal(c32.view(np.uint32), b32.view(np.uint32))
    assert cst[0] > 0 and not bst[[0, 1, 2, 3, 4, 5, 8, 9, 10, 11]].any()  # the baseline counts no tests


def test_deep_scene_reaches_past_the_lds_stack():
    """DEEP (scenes.deep_scene): the per-lane traversal's stack goes past the device's 32 LDS entries, so the
    -m gpu concurrency test really exercises the HBM overflow stack."""
    spec = scenes.config("DEEP")
    o = oracle.Scene(spec)
    tlas, blas = o.tlas_info(), o.blas_info(0)
    assert int(tlas[3]) + 1 + int(blas[3]) > 32
    oracle.max_stack_reached()
    o.render_spec(spec, nthreads=1, schedule=1)
    assert oracle.max_stack_reached() > 32


def test_fullsize_float64_crosscheck_fixture():
    """tests/golden/fullsize_numpy.json (make_golden.py --fullsize): evenly spaced rows of FULL-size frames of C2,
    C2F, C3, C4 and REF rendered by the oracle and by the independent float64 numpy restatement. Every pixel
    within the north-star 1e-3 bound, and float32 and float64 agree on every primary hit (no leak through the
    teapot's seams at these cameras). The oracle still renders those rows to the recorded bytes (no drift)."""
    import hashlib
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "fullsize_numpy.json")) as f:
        fx = json.load(f)
    assert {"C2", "C2F", "C3", "C4", "REF"} <= set(fx)
    for name, r in fx.items():
        assert r["linf"] < 1e-3 and r["pixels_over_bound"] == 0, name
        assert r["primary_hit_identity"]["leak"] == 0 and r["primary_hit_identity"]["extra"] == 0, name
        assert len(r["rows"]) >= (64 if name != "C4" else 32)
    for name in ("C2", "REF"):  # drift check on the two cheapest
        spec = scenes.config(name)
        rows = np.asarray(fx[name]["rows"], np.uint32)
        o8, _, _ = oracle.Scene(spec).render_spec(spec, rows=rows, nthreads=8, schedule=1)
        assert hashlib.sha256(o8.tobytes()).hexdigest() == fx[name]["oracle_rows_rgba8_sha256"], name


def test_seam_watertightness_probe_fixture():
    """tests/golden/seam_leaks.json (make_golden.py --seams): rays aimed at the teapot's 1,036 seam edges, float32
    Moller-Trumbore over the oracle's BVH (the GPU's arithmetic) against the float64 brute force. The
    counts are reproduced here from scratch (float32 leaks are a property of the pinned intersection test, DXR's
    is watertight: DESIGN §5)."""
    import json
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_golden
    with open(os.path.join(os.path.dirname(__file__), "golden", "seam_leaks.json")) as f:
        fx = json.load(f)
    path = os.path.join(os.path.dirname(__file__), "golden", "seam_leaks.json")
    before = open(path).read()
    try:
        make_golden.seam_leaks()
        now = json.load(open(path))
    finally:
        with open(path, "w") as f:
            f.write(before)
    for k in ("seam_edges", "rays", "hit64", "hit32", "leaks", "extra32", "same_triangle"):
        assert now[k] == fx[k], k
    assert fx["seam_edges"] == 1036 and 0 < fx["leaks"] < fx["rays"] // 10
    # ceiling: the shipped triangle test (fused cross products, unfused dots, rt_device.hpp mt_cross /
    # mt_dot) leaks 1,832 of the 66,304 edge rays; a change of that arithmetic may not leak more (regenerating the
    # fixture does not lift this bound; unfused products gave 1,727, fused dots 2,514: profiles/r03_ab_mt_fma.txt)
    assert now["leaks"] <= 1832 and fx["leaks"] <= 1832


def _stress_cases():
    """The two frames the round-5 stress run (tools/stress.py) found where the packet walk took a float32
    Moller-Trumbore false positive the per-ray walk never tests: a grazing ray just outside a triangle corner
    (float64 barycentrics about -1e-4), its own slab test rejecting the triangle's box while other lanes of its packet
    entered it. DEGEN (a sliver across the soup's box) and C4 with its instances moved as a per-frame update."""
    import math
    deg = scenes.degenerate_scene().with_size(80, 44)
    deg.camera = ((-4.14559724980539, 7.847480531308231, 21.095124369916352), (0.0, 1.0, 1.0), (0.0, 1.0, 0.0))
    c4 = scenes.config("C4").with_size(960, 540)
    c4.camera = ((-11.381945623573028, 13.932030315755242, 22.76952599027979), (0.0, 1.0, 0.0), (0.0, 1.0, 0.0))
    inst = []
    for (m, x, iid, hg) in c4.instances:
        x = np.array(x, np.float32).copy()
        if hg == 0:
            x[7] += 0.25 * math.sin(0.3 * 4 + 0.7 * iid)
        inst.append((m, x, iid, hg))
    c4.instances = inst
    return [("DEGEN", deg, (26, 30)), ("C4moved", c4, (374, 411))]


@pytest.mark.parametrize("case", [0, 1])
def test_packet_takes_only_its_own_boxes_hits(case):
    """Each lane of a packet may only take hits of triangles whose slot box its own slab test accepted
    (packet_tri's own mask): the packet image then equals the per-ray image on the stress cases too. The
    pixel in question is lit in both (the per-ray walk's answer; the unmasked packet walk had it black)."""
    name, spec, (y, x) = _stress_cases()[case]
    o = oracle.Scene(spec)
    a8, a32, _ = o.render_spec(spec, nthreads=8, schedule=1)
    b8, b32, _ = o.render_spec(spec, nthreads=8, schedule=0)
    assert np.array_equal(a8, b8) and np.array_equal(a32, b32), name
    assert b32[y, x, 0] > 0.5, (name, b32[y, x])
