"""The packet walk's triangle acceptance (rt_device.hpp moller_trumbore_flat, RT_FLAT_UV2) drops the reference
predicate's u <= 1 and tests min(u, v) >= 0 instead of u >= 0 and v >= 0. That is the same predicate for every
pair of float32 values, which this test checks exhaustively over the special values (+-0, +-inf, NaN, the
neighbours of 0 and 1, denormals) and over random pairs near the triangle's edges, in float32 arithmetic
(np.fmin is C's fminf: a NaN operand yields the other one, as v_min_f32 does)."""
import numpy as np


def _reference(u, v):
    return (u >= 0) & (u <= 1) & (v >= 0) & ((u + v) <= 1)


def _reduced(u, v):
    return (np.fmin(u, v) >= 0) & ((u + v) <= 1)


def _specials():
    f = np.float32
    one, zero = f(1), f(0)
    vals = [zero, -zero, one, -one, f(0.5), np.inf, -np.inf, np.nan, np.finfo(f).tiny, -np.finfo(f).tiny,
            f(1e-45), f(-1e-45), np.nextafter(one, f(2)), np.nextafter(one, zero), np.nextafter(zero, one),
            np.nextafter(zero, -one), f(2), f(1e30), f(-1e30), np.nextafter(f(0.5), one), np.nextafter(f(0.5), zero)]
    return np.array(vals, np.float32)


def test_reduced_acceptance_equals_reference_on_special_values():
    s = _specials()
    u, v = np.meshgrid(s, s)
    with np.errstate(invalid="ignore", over="ignore"):
        assert np.array_equal(_reference(u, v), _reduced(u, v))


def test_reduced_acceptance_equals_reference_near_the_edges():
    rng = np.random.default_rng(0x5EED)
    n = 2_000_000
    # u in [-0.01, 1.01], v = 1 - u + a few ulps either way: pairs on and around the u + v = 1 edge and the axes
    u = rng.uniform(-0.01, 1.01, n).astype(np.float32)
    v = (np.float32(1) - u).astype(np.float32)
    v = (v.view(np.int32) + rng.integers(-3, 4, n).astype(np.int32)).view(np.float32)
    w = rng.uniform(-1e-6, 1e-6, n).astype(np.float32)
    for a, b in ((u, v), (v, u), (u, w), (w, u), (w, w)):
        with np.errstate(invalid="ignore", over="ignore"):
            assert np.array_equal(_reference(a, b), _reduced(a, b))
