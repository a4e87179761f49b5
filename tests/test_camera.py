"""Camera: Manipulator::setLookat/update == glm::lookAtRH (manipulator.cpp:26-32,305-314) and the
256-B camera constant buffer of UpdateCameraBuffer (D3D12HelloTriangle.cpp:1144-1170).

Golden: tests/golden/camera_glm.json, produced by compiling the reference's vendored glm
(oracle/ref_glm_camera.cpp -> oracle/_ref/glm_camera; script tests/golden/make_golden.py).
"""
import json
import os

import numpy as np
import pytest

import realtimeraytracing_gradproject_amd as rt
import oracle

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "camera_glm.json")))


@pytest.mark.parametrize("case", GOLD["lookat"], ids=lambda c: str(c["eye"]))
def test_lookat_bitwise_equals_reference_glm(case):
    got = rt.camera_lookat(case["eye"], case["center"], case["up"])
    assert got.view(np.uint32).tolist() == case["view_bits"]
    ora = oracle.camera_lookat(case["eye"], case["center"], case["up"])
    assert ora.view(np.uint32).tolist() == case["view_bits"]


def test_reference_view_matches_survey_value():
    v = rt.camera_lookat((1.5, 1.5, 1.5), (0, 0, 0), (0, 1, 0))
    expect = [0.707107, -0.408248, 0.57735, 0, 0, 0.816497, 0.57735, 0, -0.707107, -0.408248, 0.57735, 0, 0, 0,
              -2.59808, 1]  # SURVEY.md §8c (getMatrix of the compiled reference manipulator)
    assert np.allclose(v, expect, atol=5e-6)


@pytest.mark.parametrize("W,H", [(1280, 720), (1920, 1080), (512, 512), (3840, 2160), (97, 13)])
def test_camera_buffer(W, H):
    view = rt.camera_lookat((1.5, 1.5, 1.5), (0, 0, 0), (0, 1, 0))
    cb = rt.camera_buffer(view, W, H)
    assert np.array_equal(cb[:16], view)
    # XMMatrixPerspectiveFovRH(45 deg, W/H, 0.1, 1000), row-major XMMATRIX memory
    h = 1.0 / np.tan(np.deg2rad(22.5))
    P = cb[16:32].reshape(4, 4)
    assert np.isclose(P[1, 1], h, rtol=1e-6) and np.isclose(P[0, 0], h / (W / H), rtol=1e-6)
    assert np.isclose(P[2, 2], 1000 / (0.1 - 1000), rtol=1e-6) and P[2, 3] == -1.0
    assert np.isclose(P[3, 2], 1000 * 0.1 / (0.1 - 1000), rtol=1e-6) and P[3, 3] == 0.0
    for k in (0, 1):
        M = cb[16 * k:16 * k + 16].reshape(4, 4).astype(np.float64)
        Minv = cb[32 + 16 * k:48 + 16 * k].reshape(4, 4).astype(np.float64)
        assert np.allclose(M @ Minv, np.eye(4), atol=2e-6)
    # the oracle computes the inverses independently (Gauss-Jordan vs cofactors, both in double)
    ocb = oracle.camera_buffer(view, W, H)
    assert np.allclose(cb, ocb, rtol=1e-7, atol=1e-9)


def test_ray_directions_closed_form():
    """projInv * (x, -y, 1, 1) has xyz = (x tan(fov/2) aspect, -y tan(fov/2), -1)."""
    W, H = 1280, 720
    cb = rt.camera_buffer(rt.camera_lookat((0, 0, 0), (0, 0, -1), (0, 1, 0)), W, H)
    Pinv = cb[48:64].reshape(4, 4).T.astype(np.float64)  # HLSL column-major read
    x, y = 0.3, -0.7
    r = Pinv @ np.array([x, -y, 1, 1])
    t = np.tan(np.deg2rad(22.5))
    assert np.allclose(r[:3], [x * t * W / H, -y * t, -1.0], atol=1e-6)
