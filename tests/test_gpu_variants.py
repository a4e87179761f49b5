"""Every non-default code-shape knob left in the trace kernel (rt_device.hpp / rt_trace.hip) is built by `make` as a
library variant (Makefile VARIANTS, lib/variants/<name>/librtamd.so) and rendered here against the oracle, so no
compiled-out kernel path stays untested. Among them the north star's "wavefront ballot /
prefix-sum ray compaction" designs (measured slower than the shipped packet walk and kept as
variants): the workgroup shadow-ray compaction (RT_SHADOW_COMPACT: a ballot per wave, the waves' counts through
LDS, the rays compacted by prefix + mbcnt into one packet) and the per-lane subtree hand-off (RT_HYBRID_T: the
lanes wanting a BLAS node ranked by mbcnt of the ballot into a per-wave LDS stack). Images must equal the
oracle's bit for bit; the traversal counters too where the variant keeps the shipped packet composition."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import realtimeraytracing_gradproject_amd as rt  # noqa: E402
from realtimeraytracing_gradproject_amd import scenes  # noqa: E402

import oracle  # noqa: E402

VDIR = os.path.join(os.path.dirname(rt.LIB_PATH), "variants")
VARIANTS = ["n1", "n1root", "rays2", "alt", "wavetimes", "ldstop"]
# the shipped walk's packets (counters equal the oracle's packet emulation): the code-shape variant, except its
# multi-sample frames (RT_MS_WIDE: 8 x 2-pixel tiles of 4 sample lanes instead of 4 x 4); the LDS-staged node loads
SAME_PACKETS = {"alt", "ldstop"}
# (config, size): Lambert + shadow (C2 from inside the teapot, C2F framed, C4 64 instances), multi-sample (C5),
# the reference scene (PBR, plane shadow ray) with and without reflection chains, the degenerate scene
CASES = [("C2", (192, 108)), ("C2F", (200, 101)), ("C4", (256, 136)), ("C5", (64, 36)), ("REF", (96, 54)),
         ("REFL", (64, 37)), ("DEGEN", (96, 54))]
_LIBS = {}
_ORACLE = {}


def variant(name):
    if name not in _LIBS:
        path = os.path.join(VDIR, name, "librtamd.so")
        assert os.path.exists(path), f"{path} missing: `make` builds the variants (no fallback)"
        _LIBS[name] = rt._load(path)
    return _LIBS[name]


def oracle_frame(name, size):
    if (name, size) not in _ORACLE:
        spec = scenes.config(name).with_size(*size) if name != "DEGEN" else scenes.degenerate_scene().with_size(*size)
        _ORACLE[(name, size)] = (spec,) + oracle.Scene(spec).render_spec(spec, nthreads=8)
    return _ORACLE[(name, size)]


@pytest.mark.parametrize("name,size", CASES)
@pytest.mark.parametrize("var", VARIANTS)
def test_variant_frames_equal_oracle(var, name, size):
    spec, o8, o32, ost = oracle_frame(name, size)
    c = rt.Context(0, library=variant(var))
    scenes.upload(c, spec)
    c.set_stats(True)
    c.stats_reset()
    out8 = torch.empty((spec.height, spec.width, 4), dtype=torch.uint8, device="cuda")
    # the wave-clock variant writes its records into the float output: one slot (16 B) per wave
    nf = max(spec.height * spec.width, 1 << 16)
    out32 = torch.zeros((nf, 4), dtype=torch.float32, device="cuda")
    c.dispatch(spec.width, spec.height, out8, out32, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    s = c.stats()
    assert np.array_equal(out8.cpu().numpy(), o8), f"{var} {name}: RGBA8 differs from the oracle"
    if var == "wavetimes":
        rec = out32.view(torch.int32).cpu().numpy()[:, :2].astype(np.int64)
        live = rec[(rec[:, 0] != 0) | (rec[:, 1] != 0)]
        assert len(live) > 0 and ((live[:, 1] - live[:, 0]) % (1 << 32) < 10_000_000).all()
    else:
        assert np.array_equal(out32[:spec.height * spec.width].cpu().numpy().reshape(o32.shape), o32), \
            f"{var} {name}: float frame differs"
    # every variant traces the same rays; the packet composition decides the traversal counters
    assert [s["primary_rays"], s["shadow_rays"], s["reflection_rays"]] == [int(ost[0]), int(ost[1]), int(ost[8])]
    if var in SAME_PACKETS and spec.spp == 1:
        keys = ["aabb_tests", "tri_tests", "instance_entries", "node_fetches", "tri_fetches", "instance_fetches"]
        assert [s[k] for k in keys] == [int(x) for x in list(ost[2:5]) + list(ost[9:12])], f"{var} {name}"
    assert s["stack_overflows"] == 0
    # the adaptive tile balance (frames 2 and 3 of a shape run its work list) renders the same image
    c.set_stats(False)
    for _ in range(3):
        c.dispatch(spec.width, spec.height, out8, None, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(out8.cpu().numpy(), o8), f"{var} {name}: frame with the tile balance differs"
    c.close()
