"""A short seeded stress run (tools/stress.py, ~25 s): randomised scenes, sizes, tile-balance modes, streams, moving
cameras, per-frame TLAS updates and loopback tiled-loop episodes, with schedule, loopback and oracle checks as it
goes. The long runs are in profiles/r05_stress_seed{1,2}.log."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_short_stress_run_is_clean():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "stress.py"), "--minutes", "0.4", "--seed", "3"],
                       capture_output=True, text=True, timeout=110)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    last = json.loads(lines[-1])
    assert last.get("stress") == "ok", last
    assert last["episodes"] > 50 and last["oracle_checks"] > 20 and last["schedule_checks"] > 50, last
