#!/usr/bin/env python3
"""Per-level triangular-solve schedule probe for the configs[4] hierarchy: the Gauss-Seidel factor
triu(A_l) of every SA level of -FD side^2 (numLevels=5, as bench.py's configs4 key), each schedule
forced in turn and timed (3 applies after one warm apply). Development tool only.

    python tools/level_sched_probe.py --side 8192
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
    ap.add_argument("--side", type=int, default=8192)
    ap.add_argument("--levels", type=int, default=5)
    args = ap.parse_args()
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear import SmoothedAggregationMLHierarchy, TriangularSolveChain
    A = -psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, args.side).to_scipy()
    t0 = time.perf_counter()
    h = SmoothedAggregationMLHierarchy(A, numLevels=args.levels)
    print(json.dumps({"setup_s": time.perf_counter() - t0}), flush=True)
    for lev in range(1, args.levels - 1):
        Al = h.matrix(lev).tocsr()
        U = sp.triu(Al).tocsr()
        n = U.shape[0]
        M = TriangularSolveChain(n, U=U)
        out = {"level": lev, "n": n, "nnz_U": int(U.nnz), "default": M.schedule("U")}
        v = psk.DeviceVector.from_numpy(np.random.default_rng(lev).standard_normal(n))
        ref = None
        for sched in ("syncfree", "band", "part", "grid"):
            try:
                M.schedule("U", set=sched)
            except N.PskError as e:
                out[sched + "_ms"] = None
                continue
            r = M.apply(v)
            N.check(N.lib.psk_synchronize(), "sync")
            t = time.perf_counter()
            for _ in range(3):
                M.apply(v)
            N.check(N.lib.psk_synchronize(), "sync")
            out[sched + "_ms"] = (time.perf_counter() - t) * 1e3 / 3
            rn = r.numpy() if hasattr(r, "numpy") else np.asarray(r)
            if ref is None:
                ref = rn
            else:
                out[sched + "_bitwise"] = bool(np.array_equal(rn, ref))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
