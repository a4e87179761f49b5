"""Camera manipulator: nv_helpers_dx12::Manipulator motion — mouseMove bindings,
orbit / pan / dolly / trackball / look-around, wheel, roll, the Examine/Fly/Walk/Trackball modes
and the dolly/orbit guards — replayed through the C-ABI rt_manip_* functions (host code, no GPU)
against tests/golden/manipulator.json: trajectories computed with the reference's own vendored
glm 0.9.8.5 (oracle/ref_glm_manip.cpp; src/manipulator.cpp itself includes windows/d3d12 headers
and cannot be built here). Bit-exact on eye, interest, up and the 4x4 view matrix."""
import ctypes
import json
import math
import os

import numpy as np
import pytest

import realtimeraytracing_gradproject_amd as rt

GOLD = os.path.join(os.path.dirname(__file__), "golden", "manipulator.json")


def replay(m: rt.Manipulator, e: dict) -> int:
    op, a = e["op"], e["args"]
    if op == "lookat":
        m.setLookat(a[0:3], a[3:6], a[6:9])
    elif op == "window":
        m.setWindowSize(int(a[0]), int(a[1]))
    elif op == "mouse":
        m.setMousePosition(int(a[0]), int(a[1]))
    elif op == "mode":
        m.setMode(int(a[0]))
    elif op == "roll":
        m.setRoll(a[0])
    elif op == "speed":
        m.setSpeed(a[0])
    elif op == "move":
        return m.mouseMove(int(a[0]), int(a[1]), int(a[2]))
    elif op == "motion":
        m.motion(int(a[0]), int(a[1]), int(a[2]))
    elif op == "wheel":
        m.wheel(int(a[0]))
    else:
        raise ValueError(op)
    return -1


def bits(v) -> list:
    return np.asarray(v, np.float32).view(np.uint32).tolist()


def sequences():
    with open(GOLD) as f:
        return json.load(f)["sequences"]


@pytest.mark.parametrize("seq", sequences(), ids=lambda s: s["name"])
def test_trajectory_bit_exact(seq):
    m = rt.Manipulator()
    for i, e in enumerate(seq["events"]):
        ret = replay(m, e)
        eye, center, up = m.getLookat()
        where = f"{seq['name']} event {i} {e['op']}{e['args']}"
        assert ret == e["ret"], where
        assert bits(eye) == e["eye"], where
        assert bits(center) == e["center"], where
        assert bits(up) == e["up"], where
        assert bits(m.getMatrix()) == e["matrix"], where


def test_golden_covers_every_action_and_mode():
    acts, modes, ops = set(), {0}, set()
    for s in sequences():
        for e in s["events"]:
            ops.add(e["op"])
            if e["op"] == "move":
                acts.add(e["ret"])
            if e["op"] == "mode":
                modes.add(int(e["args"][0]))
    assert acts == {0, 1, 2, 3, 4}
    assert modes == {0, 1, 2, 3}
    assert {"lookat", "window", "mouse", "mode", "roll", "speed", "move", "motion", "wheel"} <= ops


def test_defaults_and_layout():
    assert ctypes.sizeof(rt.rt_manipulator) == 132
    m = rt.Manipulator()  # manipulator.h:124-144
    eye, c, up = m.getLookat()
    assert eye.tolist() == [10, 10, 10] and c.tolist() == [0, 0, 0] and up.tolist() == [0, 1, 0]
    assert m.getSpeed() == 30 and m.getMode() == rt.Manipulator.Examine and m.getRoll() == 0
    assert m.getWidth() == 1 and m.getHeight() == 1
    assert np.array_equal(m.getMatrix(), rt.camera_lookat((10, 10, 10), (0, 0, 0), (0, 1, 0)))


def test_orbit_keeps_distance_and_full_width_is_a_turn():
    """Orbit about the interest point preserves the eye distance; a drag of the full window width
    is one full turn about up (manipulator.cpp:350-352)."""
    m = rt.Manipulator()
    m.setWindowSize(1000, 1000)
    m.setLookat((0, 0, 5), (0, 0, 0), (0, 1, 0))
    m.setMousePosition(0, 500)
    assert m.mouseMove(250, 500, rt.Manipulator.inputs(lmb=True)) == rt.Manipulator.Orbit
    eye, _, _ = m.getLookat()
    assert abs(float(np.linalg.norm(eye)) - 5.0) < 1e-5
    assert np.allclose(eye, (5, 0, 0), atol=1e-5)  # quarter width -> quarter turn about +y
    m.mouseMove(1000, 500, rt.Manipulator.inputs(lmb=True))  # 0 -> 1000 in total: one full turn
    eye, _, _ = m.getLookat()
    assert np.allclose(eye, (0, 0, 5), atol=1e-4)


def test_pan_moves_eye_and_interest_together_and_dolly_never_crosses():
    m = rt.Manipulator()
    m.setWindowSize(100, 100)
    m.setLookat((0, 0, 10), (0, 0, 0), (0, 1, 0))
    m.setMousePosition(50, 50)
    m.mouseMove(60, 50, rt.Manipulator.inputs(mmb=True))
    eye, c, _ = m.getLookat()
    assert np.allclose(eye - c, (0, 0, 10), atol=1e-5) and c[0] < 0 and c[1] == 0
    for y in range(40, -400, -10):  # rmb drags upward: dolly in, step shrinking with distance
        m.mouseMove(60, y, rt.Manipulator.inputs(rmb=True))
        eye, c, _ = m.getLookat()
        assert (eye - c)[2] > 0
    assert m.getRoll() == 0
    m.setRoll(math.pi / 2)
    v = m.getMatrix().reshape(4, 4)  # column-major: v[c][r]
    assert abs(float(v[0][1]) + 1.0) < 1e-6 or abs(float(v[0][1]) - 1.0) < 1e-6


def test_wheel_and_unbound_buttons():
    m = rt.Manipulator()
    m.setWindowSize(640, 480)
    before = m.getMatrix()
    assert m.mouseMove(10, 10, 0) == rt.Manipulator.NoAction
    assert np.array_equal(m.getMatrix(), before)
    m.wheel(-1)  # wheel down: dolly toward the interest point
    eye, _, _ = m.getLookat()
    assert float(np.linalg.norm(eye)) < float(np.linalg.norm([10, 10, 10]))
