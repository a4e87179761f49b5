"""bench.py's untimed autotunes on a fake backend (CPU): pick_in_flight measures 1..4 streams drawn
from ONE pool and hands back the very streams it measured. The fake backend's frame cost depends on the stream set, the way a HIP runtime that maps two
streams onto one hardware queue would make it."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class _S:
    def __init__(self, q):
        self.q = q  # the hardware queue this stream landed on


class FakeBackend:
    multi_stream = True

    def __init__(self, queues, frame_s=0.0004):
        self._queues = list(queues)  # queue of each stream in creation order
        self.frame_s = frame_s
        self.pending = {}
        self.tile = 8

    def stream(self):
        return _S(self._queues.pop(0))

    def zeros(self, shape):
        return bytearray(1)

    def dispatch(self, buf, rows, stream):
        # frames on distinct queues overlap: the cost of a batch is the busiest queue's
        self.pending[stream.q] = self.pending.get(stream.q, 0) + 1

    def synchronize(self):
        if self.pending:
            time.sleep(self.frame_s * max(self.pending.values()))
        self.pending = {}


def test_pick_in_flight_returns_measured_streams():
    # streams 0 and 1 share queue 0: two streams gain nothing; with four, the busiest queue runs
    # half the frames
    be = FakeBackend([0, 0, 1, 2])
    s, ms, streams = bench.pick_in_flight(be, 8, 8, None, frames=8, rounds=1)
    assert s == 4 and [x.q for x in streams] == [0, 0, 1, 2]
    assert ms[4] < ms[2] and set(ms) == {1, 2, 3, 4}


def test_pick_in_flight_keeps_one_without_streams():
    class NoStreams:
        pass
    assert bench.pick_in_flight(NoStreams(), 8, 8, None) == (1, None, None)


def test_pick_in_flight_near_ties_take_more_streams(monkeypatch):
    """Measured times within 1 % of the fastest count as a tie: the autotune then takes the most frames in flight
    (a short timed region runs two streams' frames in lockstep pairs)."""
    be = FakeBackend([0, 1, 2, 3])
    fake = {1: 0.130, 2: 0.1150, 3: 0.1155, 4: 0.1170}
    times = iter([])

    def fake_counter():
        return next(times)
    # one round over choices 1..4: each measurement is two perf_counter reads (start, end)
    seq = []
    for n in (1, 2, 3, 4):
        seq += [0.0, fake[n] * 16 / 1e3]
    times = iter(seq)
    monkeypatch.setattr(bench.time, "perf_counter", fake_counter)
    s, ms, streams = bench.pick_in_flight(be, 8, 8, None, frames=16, rounds=1)
    assert s == 3 and len(streams) == 3  # 3 is within 1 % of 2's 0.1150; 4 is not
    assert ms[2] == 0.115 and ms[3] == 0.1155
