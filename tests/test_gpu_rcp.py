"""rt::rcp_exact (rt_device.hpp), the trace kernel's 1 / det in the triangle test: v_rcp_f32 + one fused Newton
step where the exponent is in [20, 234], the IEEE division for the wave otherwise. It must give the bits of
`1.0f / x` -- what the oracle computes on the CPU -- for EVERY float. tools/bin/recip_check (built by `make`)
checks all 2^32 patterns on the GPU in about a second; the frame-parity tests then hold by construction."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "bin", "recip_check")


def _run(*args):
    assert os.path.exists(EXE), "tools/bin/recip_check missing: run make"
    r = subprocess.run([EXE, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    counts = {m.group(1): int(m.group(2)) for m in re.finditer(r"^(\w) \(.*?\): (\d+) mismatches", r.stdout, re.M)}
    assert set(counts) == {"A", "B", "E"}, r.stdout
    return counts


def test_rcp_exact_equals_ieee_division_for_every_float():
    c = _run("0", "255")
    assert c["E"] == 0


def test_fast_path_exact_on_its_whole_range():
    c = _run("20", "234")
    assert c["A"] == 0 and c["E"] == 0
