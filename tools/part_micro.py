#!/usr/bin/env python3
"""Hop-latency microbenchmark of the triangular-solve schedules (development probe, GPU).

    python tools/part_micro.py

Unit-diagonal-free lower factors with fixed dependency offsets in the natural order (row i depends
on i-d for every d in the set), so every dependency level costs one hand-off: inside a strip for
the partitioned schedule (LDS), across waves for sync-free. Prints us per level for each schedule.
"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def factor(n, offs):
    i = np.arange(n)
    rows = np.concatenate([i[d:] for d in offs])
    cols = np.concatenate([i[:-d] for d in offs])
    vals = np.concatenate([np.full(n - d, -0.4 / len(offs)) for d in offs])
    return (sp.csr_matrix((vals, (rows, cols)), shape=(n, n)) + sp.diags(np.full(n, 1.5))).tocsr()


def main():
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear import TriangularSolveChain
    cases = [("chain1", 65536, (1,)), ("chain64", 1 << 20, (64,)), ("chain64+1", 1 << 18, (1, 64)),
             ("chain256", 1 << 22, (256,))]
    if os.environ.get("PART_MICRO_CASES"):
        cases = [c for c in cases if c[0] in os.environ["PART_MICRO_CASES"].split(",")]
    for name, n, offs in cases:
        L = factor(n, offs)
        os.environ["PSK_TRISOLVE_PART"] = "1"
        M = TriangularSolveChain(n, L=L)
        del os.environ["PSK_TRISOLVE_PART"]
        levels = M.device_info()["levels_l"]
        v = np.random.default_rng(1).standard_normal(n)
        out = {"case": name, "n": n, "levels": levels}
        res = {}
        for sched in ("part", "syncfree"):
            M.schedule("L", set=sched)
            M.apply(v)
            ts = []
            for _ in range(3):
                N.check(N.lib.psk_synchronize(), "sync")
                t0 = time.perf_counter()
                res[sched] = M.apply(v)
                N.check(N.lib.psk_synchronize(), "sync")
                ts.append((time.perf_counter() - t0) * 1e3)
            out[sched + "_ms"] = sorted(ts)[1]
            out[sched + "_us_per_level"] = out[sched + "_ms"] * 1e3 / levels
        out["bit_identical"] = bool(np.array_equal(res["part"], res["syncfree"]))
        if hasattr(N.lib, "psk_part_trace_read") and n <= (1 << 17):   # -DPSK_PART_PROF build
            import ctypes
            M.schedule("L", set="part")
            M.apply(v)
            N.check(N.lib.psk_synchronize(), "sync")
            tr = np.zeros(8 * n, np.uint64)
            N.lib.psk_part_trace_read(tr.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(n))
            ph = tr.reshape(n, 8).astype(np.int64)
            # strip 0's positions (workgroup 0): in these factors position order is natural order, so
            # consecutive positions of a chain1 strip are consecutive hops (row k needs row k-1)
            R = n // 256
            k = np.arange(1, R)
            prod_done, start = ph[k - 1, 5], ph[k, 0]
            ready = np.maximum(start, prod_done)   # the consumer's turn AND the producer's value written
            med = lambda a: float(np.median(a))
            out["phases_cycles_median"] = {
                "turn_after_producer": med(start - prod_done),       # < 0: the consumer waited for the value
                "detect_lds": med(ph[k, 1] - ready),                  # value written -> seen by the spin
                "values_and_fma": med(ph[k, 2] - ph[k, 1]),           # remote polls + fma chain
                "row_total_dpp": med(ph[k, 3] - ph[k, 2]),
                "quotient": med(ph[k, 4] - ph[k, 3]),
                "publish_issue": med(ph[k, 5] - ph[k, 4]),
                "hop_period": med(ph[k, 5] - ph[k - 1, 5]),
                "spin_waited_frac": float(np.mean(ph[k, 6])), "spins_median": med(ph[k, 7])}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
