#!/usr/bin/env python3
"""Larger golden case, run through the REFERENCE itself (build container only).

FDLaplacian2D(-1, 1, 1024) (n = 1,048,576) + PCG with Jacobi, tau = 1e-8,
b = A @ default_rng(12345).random(n). Stores the iteration count, the full
residual history and a head/hash of b (x_exact is regenerated from the seed).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_large.py
"""
import hashlib
import os
import sys
import time

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg                      # noqa: E402  (installs the stand-ins, imports the reference)
from oracle import fdlap, krylov              # noqa: E402


def main(m=1024):
    t = time.time()
    A = mg.ref_fd2d(-1.0, 1.0, m)             # reference DOK generator (slow, ~1 min)
    ip, ix, dt = fdlap.fd_laplacian_2d_arrays(-1.0, 1.0, m)
    assert np.array_equal(A.indptr, ip) and np.array_equal(A.indices, ix) and np.array_equal(A.data, dt)
    print("generator ok (%.0f s)" % (time.time() - t))
    x = np.random.default_rng(12345).random(m * m)
    b = mg.ref_mvmult(A, x)
    res, hist = mg._run_ref("pcg", A, b, 4000, 1e-8, True, True)
    orc = krylov.pcg(A, b, maxiter=4000, tau=1e-8, precond=krylov.jacobi_form(A))
    mg._check_same("fd%d" % m, res, hist, orc)
    print("reference PCG+Jacobi m=%d: iters=%d (%.0f s)" % (m, res.iters(), time.time() - t))
    sens = mg.sensitivity("pcg", A, b, 4000, 1e-8, True, True, hist, res.soln(), seeds=3)
    print("sensitivity", sens)
    np.savez_compressed(os.path.join(HERE, "large_fd%d.npz" % m), iters=np.int64(res.iters()), hist=hist,
                        b_head=b[:4096], b_sha256=np.array(hashlib.sha256(b.tobytes()).hexdigest()),
                        resid=np.float64(res.resid()), m=np.int64(m),
                        sens_hist=np.float64(sens["hist_over_normb"]), sens_x=np.float64(sens["x_rel"]),
                        soln_head=res.soln()[:4096], soln_norm=np.float64(np.linalg.norm(res.soln())))


if __name__ == "__main__":
    main()
