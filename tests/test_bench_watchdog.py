"""bench.py's liveness watchdog (round 6): the progress counter advances only when work completes, the
heartbeat line reports the counter and its age, and a phase whose counter stalls past its limit ends the run
with exit code 3 and the phase named. CPU only: a fake clock drives Liveness directly."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def _live(**kw):
    import bench
    clk, lines, exits = Clock(), [], []
    lv = bench.Liveness(gpu_stall_s=150.0, host_stall_s=420.0, beat_s=30.0, clock=clk, write=lines.append,
                        exit_fn=exits.append, **kw)
    return lv, clk, lines, exits


def test_progress_resets_the_stall_clock():
    lv, clk, lines, _ = _live()
    lv.phase("headline")
    assert lines[-1].startswith("bench: headline (gpu phase")
    for _ in range(10):        # a libpsk call returns every 100 s: never stalled
        clk.t += 100.0
        assert lv.stalled() is None
        lv.tick("psk_pcg")
    assert lv.count == 11      # the phase change counts as one advance
    clk.t += 149.0
    assert lv.stalled() is None
    assert "progress 11, last: psk_pcg 149 s ago" in lv.line()


def test_gpu_phase_stall_is_reported():
    lv, clk, _, _ = _live()
    lv.phase("strong_scaling_16384")
    lv.tick("psk_pcg")
    clk.t += 151.0
    msg = lv.stalled()
    assert msg is not None and "WATCHDOG" in msg and "'strong_scaling_16384'" in msg and "gpu phase" in msg
    assert "last advance: psk_pcg" in msg and "exiting with code 3" in msg


def test_host_phase_has_the_longer_limit():
    lv, clk, _, _ = _live()
    lv.phase("configs2_gmres30_ilut (host SuperLU ILUT first)", "host")
    clk.t += 400.0               # one long spilu call: no tick, still within the host limit
    assert lv.stalled() is None
    clk.t += 30.0
    assert "host phase" in lv.stalled()
    lv.phase("configs2_gmres30_ilut: device solves")   # back to GPU work: the clock restarts
    assert lv.stalled() is None


def test_watchdog_thread_exits_on_stall():
    """The thread: heartbeat lines while work advances, then the stuck phase and exit code 3, once."""
    import threading
    import time
    import bench
    lines, exits = [], []
    done = threading.Event()

    def ex(code):
        exits.append(code)
        done.set()
    lv = bench.Liveness(gpu_stall_s=0.3, host_stall_s=0.3, beat_s=0.05, write=lines.append, exit_fn=ex)
    lv.phase("headline")
    lv.start()
    for _ in range(6):            # progress: no exit
        time.sleep(0.05)
        lv.tick("psk_pcg")
    assert not exits
    assert done.wait(5.0)         # then a stall
    time.sleep(0.2)
    assert exits == [3]
    assert any("WATCHDOG" in x and "'headline'" in x for x in lines)
    assert any("progress" in x for x in lines if "WATCHDOG" not in x)


@pytest.mark.parametrize("kind", ["gpu", "host"])
def test_phase_line_names_kind(kind):
    lv, _, lines, _ = _live()
    lv.phase("x", kind)
    assert "(%s phase" % kind in lines[-1]
