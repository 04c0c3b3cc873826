#!/usr/bin/env python3
"""Lab probe: per-region wall times of the bench's headline solve in sequences (why is the first timed region
slower?). One process, N = 10M (bench.PcgSystem), each sequence on the same system:

    python tools/region_probe.py [--side 3163] [--steps 20] [--regions 8]

Sequences: settle then warm-up W = 5 with events then regions with events (the bench's order); the same with
W = steps; no events anywhere; and regions separated by a 20 ms host sleep. Prints one JSON line each.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=3163)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--regions", type=int, default=8)
    a = ap.parse_args()
    os.environ.setdefault("PSK_NO_TORCH", "1")
    import bench
    from pysolvers_amd import _native as N
    N.check(N.lib.psk_set_device(0), "set_device")
    s = bench.PcgSystem(N, a.side, None, 1)

    def seq(name, warm, events, gap=0.0, settle=True):
        if settle:
            s.run(s.settle_iters(), False)
        if warm:
            s.run(warm, events)
        out = []
        for _ in range(a.regions):
            if gap:
                time.sleep(gap)
            N.check(N.lib.psk_synchronize(), "sync")
            t0 = time.perf_counter()
            r = s.run(a.steps, events)
            t1 = time.perf_counter()
            N.check(N.lib.psk_synchronize(), "sync")
            t2 = time.perf_counter()
            out.append({"it_s": round(a.steps / (t2 - t0), 1), "call_ms": round((t1 - t0) * 1e3, 3),
                        "spmv_us": round(r.spmv_ms * 1e3, 2)})
        print(json.dumps({"seq": name, "regions": out}), flush=True)

    seq("bench_order", 5, True)
    seq("bench_order_again", 5, True)
    seq("warm_eq_steps", a.steps, True)
    seq("no_events", 5, False)
    seq("gap_20ms", 5, True, gap=0.02)
    seq("no_settle", 5, True, settle=False)
    s.free()


if __name__ == "__main__":
    main()
