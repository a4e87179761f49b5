"""Seeded random scenes on the CPU oracle (tests/random_scenes.py): the packet emulation (the device's default
schedule) renders the per-ray schedule's image bit for bit (its lanes take hits only in boxes their own slab tests
accept), and on these seeds both equal brute force (every triangle of every instance tested per ray) where
the scene is small enough for it — brute force alone can take float32 Moller-Trumbore false positives of rays grazing
a triangle corner outside its box, which none of these seeds has. Random meshes, instance transforms (rotated,
non-uniformly scaled, mirrored, translate-only), hit groups, lights, materials, cameras, shading modes and 1 / 4 spp:
the cases the fixed configs do not reach."""
import numpy as np
import pytest

import oracle
from random_scenes import random_scene

SEEDS = list(range(16))


@pytest.mark.parametrize("seed", SEEDS)
def test_random_scene_schedules_and_brute_force_agree(seed):
    spec = random_scene(seed)
    o = oracle.Scene(spec)
    a8, a32, _ = o.render_spec(spec, nthreads=8, schedule=0)
    b8, b32, _ = o.render_spec(spec, nthreads=8, schedule=1)
    assert np.array_equal(a32, b32) and np.array_equal(a8, b8), f"seed {seed}: packet emulation != per-ray"
    ntri = [m[1].size // 3 if m[1] is not None else m[0].shape[0] // 3 for m in spec.meshes]
    work = sum(ntri[m] for (m, *_) in spec.instances)  # triangles a brute-force ray tests
    if work > 60000:
        return  # brute force over this many triangles per ray: covered by the smaller seeds
    small = spec.with_size(48, 32)
    c8, c32, _ = o.render_spec(small, nthreads=8, schedule=0)
    d8, d32, _ = o.render_spec(small, nthreads=8, brute_force=True)
    assert np.array_equal(c32, d32) and np.array_equal(c8, d8), f"seed {seed}: BVH walk != brute force"
