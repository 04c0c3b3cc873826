#!/usr/bin/env python3
"""Lab probe: one SA level's Gauss-Seidel factor triu(A_k) (ClassicSmoothers.py:33) under each triangular-solve
schedule, with the partitioned schedule built at several strip counts (PSK_PART_STRIPS, one process each).

    python tools/level_probe.py [--side 8192] [--levels 5] [--level 1] [--strips 256,64,32,16] [--reps 20]

The hierarchy of -FDLaplacian2D(side) is built once on the host (SmoothedAggregationMLHierarchy, O(nnz)) and
A_k cached in /tmp; each child creates the chain with PSK_TRISOLVE_PART=1 and prints one JSON line of median
solve ms per schedule (and the dependency levels).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import scipy.sparse as sp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def child(path, reps):
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear import TriangularSolveChain
    z = np.load(path)
    A = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=tuple(z["shape"]))
    U = sp.triu(A).tocsr()
    M = TriangularSolveChain(A.shape[0], U=U)
    v = psk.DeviceVector.from_numpy(np.random.default_rng(1).standard_normal(A.shape[0]))
    out = psk.DeviceVector(A.shape[0])
    res = {"n": A.shape[0], "levels": M.device_info()["levels_u"], "planned": M.schedule("U")["schedule"]}
    ref = None
    for sched in ("syncfree", "part", "band", "levels"):
        try:
            M.schedule("U", set=sched)
        except N.PskError:
            continue
        ts = []
        for _ in range(reps + 1):
            N.check(N.lib.psk_synchronize(), "sync")
            t = time.perf_counter()
            N.check(N.lib.psk_prec_apply(M.device_handle, A.shape[0], v._p, out._p, N.PSK_DEVICE), "apply")
            ts.append(time.perf_counter() - t)
        y = out.numpy()
        if ref is None:
            ref = y
        res[sched + "_ms"] = float(np.median(ts[1:])) * 1e3
        res[sched + "_same_bits"] = bool(np.array_equal(y.view(np.uint64), ref.view(np.uint64)))
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=8192)
    ap.add_argument("--levels", type=int, default=5)
    ap.add_argument("--level", type=int, default=1)
    ap.add_argument("--strips", default="256,64,32,16")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--child", default="")
    ap.add_argument("--use-levels", type=int, default=0,
                    help="1: PSK_TRISOLVE_LEVELS=1 (the levels schedule) instead of the part sweep")
    a = ap.parse_args()
    if a.child:
        child(a.child, a.reps)
        return
    path = "/tmp/level_probe_%d_%d_%d.npz" % (a.side, a.levels, a.level)
    if not os.path.exists(path):
        os.environ.setdefault("PSK_NO_TORCH", "1")
        from oracle import fdlap
        from pysolvers_amd.Linear.SmoothedAggregation import SmoothedAggregationMLHierarchy
        A = -fdlap.fd_laplacian_2d(-1.0, 1.0, a.side)
        Ak = sp.csr_matrix(SmoothedAggregationMLHierarchy(sp.csr_matrix(A), numLevels=a.levels).matrix(a.level))
        np.savez(path, data=Ak.data, indices=Ak.indices, indptr=Ak.indptr, shape=np.array(Ak.shape))
    for P in (["0"] if a.use_levels else a.strips.split(",")):
        env = dict(os.environ, PSK_TRISOLVE_LEVELS="1") if a.use_levels else \
            dict(os.environ, PSK_TRISOLVE_PART="1", PSK_PART_STRIPS=P)
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", path, "--reps", str(a.reps)],
                           env=env, capture_output=True, text=True, timeout=300)
        line = p.stdout.strip().splitlines()[-1] if p.returncode == 0 and p.stdout.strip() else None
        print(json.dumps({"strips": int(P), "rc": p.returncode, "result": json.loads(line) if line else p.stderr[-600:]}),
              flush=True)
        if p.returncode != 0:
            sys.exit(p.returncode)


if __name__ == "__main__":
    main()
