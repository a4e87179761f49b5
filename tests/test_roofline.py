"""bench.py's roofline object and tools/roofline.py check (CPU): the line's achieved / peak / frac are the binding
pipe's, every pipe's achieved / peak equals its frac, and the checker refuses a line that breaks the
pairing. Counters are C2's from a STATS pass of the packet kernel (bench line r05); the profile inputs are the
committed profiles/roofline_inputs.json."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

bench = pytest.importorskip("bench")
import roofline as rl  # noqa: E402

ST = {"node_fetches": 955745, "tri_fetches": 392992, "instance_fetches": 96168, "primary_rays": 2073600,
      "aabb_tests": 224_600_000, "tri_tests": 25_100_000}


def _line(rf):
    return {"roofline": rf, "config": {"workload": "C2: teapot 1920x1080", "primary_rays": ST["primary_rays"]}}


def test_roofline_frac_is_the_bound_pipes(tmp_path):
    rf = bench.roofline("C2", ST, 1920 * 1080, 0.1168, "packet")
    assert rf["bound"] == max(rf["fracs"], key=rf["fracs"].get)
    assert rf["frac"] == rf["fracs"][rf["bound"]] == rf["pipes"][rf["bound"]]["frac"]
    assert abs(rf["achieved"] / rf["peak"] - rf["frac"]) < 2e-3
    assert 0 < rf["l2_frac"] < rf["frac"]  # issue-bound: the L2 is far from its roof
    assert rf["logical_bytes"]["bytes_per_launch"] == 24 * ST["aabb_tests"] + 36 * ST["tri_tests"] + 4 * 1920 * 1080
    p = tmp_path / "line.json"
    p.write_text(json.dumps(_line(rf)))
    assert rl.check(str(p)) == 0


def test_roofline_check_refuses_a_mismatched_frac(tmp_path):
    rf = bench.roofline("C2", ST, 1920 * 1080, 0.1168, "packet")
    rf["frac"] = rf["l2_frac"]  # the round-5 line: L2 fraction under a VALU bound
    p = tmp_path / "line.json"
    p.write_text(json.dumps(_line(rf)))
    assert rl.check(str(p)) == 1
