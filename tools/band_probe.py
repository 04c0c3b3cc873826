#!/usr/bin/env python3
"""Probe the band triangular-solve schedule on triu(-FD2D(m)) (the Gauss-Seidel factor):
time per sweep for a given number of blocks (PSK_BAND_BLOCKS) and both schedules.

    PSK_BAND_BLOCKS=1 python tools/band_probe.py --side 2048
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear import TriangularSolveChain
    m = args.side
    A = -psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m).to_scipy()
    U = sp.triu(A).tocsr()
    M = TriangularSolveChain(U.shape[0], U=U)
    v = psk.DeviceVector.from_numpy(np.random.default_rng(0).standard_normal(U.shape[0]))
    out = {"side": m, "blocks_env": os.environ.get("PSK_BAND_BLOCKS"), "info": M.schedule("U")}
    res = {}
    for sched in ("band", "syncfree"):
        M.schedule("U", set=sched)
        res[sched] = M.apply(v).numpy()
        N.check(N.lib.psk_synchronize(), "sync")
        t = time.perf_counter()
        for _ in range(args.reps):
            M.apply(v)
        N.check(N.lib.psk_synchronize(), "sync")
        out[sched + "_ms"] = (time.perf_counter() - t) * 1e3 / args.reps
    out["band_vs_syncfree_maxrel"] = float(np.max(np.abs(res["band"] - res["syncfree"])) /
                                           np.max(np.abs(res["syncfree"])))
    out["gate_env"] = os.environ.get("PSK_BAND_GATE")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
