#!/usr/bin/env python3
"""Lab probe of the dense coarse solve (pysolvers_amd/csrc/dense.hip): GEMV time over A^-1 and its error
against SuperLU, for a sparse SPD matrix of the AMG coarse level's size.

    python tools/dense_probe.py [--n 16642] [--reps 20] [--refine 0]

The matrix: a 2-D 9-point-like SPD pattern (the SA coarse operators' shape) of n unknowns. Prints one JSON
line: inversion time (rocSOLVER getrf + getri), GEMV ms per solve and GB/s over n x ld x 8 bytes, and the
max-norm relative difference to splu's solve.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16642)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--refine", type=int, default=0)
    a = ap.parse_args()
    os.environ.setdefault("PSK_NO_TORCH", "1")
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear.AMGPreconditioner import DenseInverseSolver
    n = a.n
    w = int(np.ceil(np.sqrt(n)))
    rng = np.random.default_rng(3)
    offs = [1, w - 1, w, w + 1]
    diags = [np.full(n - k, -rng.uniform(0.5, 1.0)) for k in offs]
    L = sp.diags(diags, offs, shape=(n, n))
    A = (L + L.T).tocsr()
    A = (A + sp.diags(np.asarray(-A.sum(axis=1)).ravel() + 1e-2)).tocsr()
    t0 = time.perf_counter()
    D = DenseInverseSolver(A, refine=a.refine)
    N.check(N.lib.psk_synchronize(), "sync")
    t_inv = time.perf_counter() - t0
    f = rng.standard_normal(n)
    dv = psk.DeviceVector.from_numpy(f)
    out = psk.DeviceVector(n)

    def apply():
        N.check(N.lib.psk_prec_apply(D.device_handle, n, dv._p, out._p, N.PSK_DEVICE), "apply")
    apply()
    ts = []
    for _ in range(a.reps):
        t1 = time.perf_counter()
        apply()
        ts.append(time.perf_counter() - t1)
    ms = float(np.median(ts)) * 1e3
    x = out.numpy()
    xs = spla.splu(A.tocsc()).solve(f)
    ld = (n + 7) // 8 * 8
    print(json.dumps({"n": n, "refine": a.refine, "invert_s": t_inv, "solve_ms": ms,
                      "gemv_GBps": n * ld * 8 * (1 + a.refine) / (ms * 1e-3) / 1e9,
                      "maxrel_vs_splu": float(np.max(np.abs(x - xs)) / np.max(np.abs(xs)))}), flush=True)


if __name__ == "__main__":
    main()
