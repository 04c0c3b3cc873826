#!/usr/bin/env python3
"""Per-solve fixed cost of psk_pcg at the bench's N = 10M (lab tool, not the bench).

    python tools/fixed_cost.py [--side 3163] [--reps 9] [--iters 0,1,2,4,8,20,200]

Wall time of one psk_pcg call (device-resident b and x, tau = 0, no timing events) per iteration count,
median of --reps calls after a warm-up solve; a least-squares line T(K) = a + b K over the counts >= 2 and
the excess of each count over it. Run it under `rocprofv3 --kernel-trace` as well to see where on the GPU
the fixed part goes (tools/solve_gaps.py reads that trace).
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
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--iters", default="0,1,2,4,8,20,200")
    a = ap.parse_args()
    os.environ.setdefault("PSK_NO_TORCH", "1")
    import bench
    from pysolvers_amd import _native as N
    N.check(N.lib.psk_set_device(0), "set_device")
    s = bench.PcgSystem(N, a.side, None, 1)
    s.run(20, False)
    out = {"side": a.side, "n": s.nloc, "reps": a.reps, "wall_ms": {}}
    for k in [int(v) for v in a.iters.split(",")]:
        ts = []
        for _ in range(a.reps):
            N.check(N.lib.psk_synchronize(), "sync")
            t0 = time.perf_counter()
            s.run(k, False)
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        out["wall_ms"][k] = ts[len(ts) // 2]
    ks = [k for k in out["wall_ms"] if k >= 2]
    if len(ks) >= 2:
        mk = sum(ks) / len(ks)
        mt = sum(out["wall_ms"][k] for k in ks) / len(ks)
        b = sum((k - mk) * (out["wall_ms"][k] - mt) for k in ks) / sum((k - mk) ** 2 for k in ks)
        out["fit"] = {"fixed_ms": mt - b * mk, "per_iter_ms": b}
        out["excess_over_fit_ms"] = {k: out["wall_ms"][k] - (mt - b * mk + b * k) for k in out["wall_ms"]}
    s.free()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
