#!/usr/bin/env python3
"""Golden fixtures for a DENSE ndarray A in the iterative solvers, made by running the REFERENCE itself.

The reference's mvmult sends a dense A through ``np.dot(A, x)`` (IterativeLinearSolver.py:94-106, a BLAS
dgemv); pysolvers_amd runs it as CSR with stored-order row sums, which rounds differently by a few ulps. No
fixture of make_golden.py held a dense solve, so that case was "parity unpinned" (DESIGN.md §2). This script
runs the reference's PCG and GMRES on dense matrices (DH-8 and FD 16^2 densified, a seeded SPD matrix and a
seeded non-symmetric diagonally dominant one), checks the oracle restatement against it, records the same
1-ulp sensitivity make_golden.py measures, and writes the inputs and the reference's outputs as data-only
fixtures (tests/golden/dense_*.npz + manifest_dense.json) that tests/test_gpu_parity.py holds the device to
with the solver cases' bars. Run only in the build container (the GPU box has no /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_dense.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg   # noqa: E402  (installs the PyTab/PyTimer stand-ins and imports the reference)


def _spd(n, seed):
    rng = np.random.default_rng(seed)
    B = rng.standard_normal((n, n))
    return B @ B.T / n + np.eye(n)


def _nonsym(n, seed):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((n, n)) / np.sqrt(n)
    return A + 3.0 * np.eye(n)


def main():
    cases = [
        ("pcg", "dh8", mg._dh(8).toarray(), 2000, 1e-8, True, False),
        ("pcg", "dh8", mg._dh(8).toarray(), 2000, 1e-8, True, True),
        ("pcg", "fd16", mg.ref_fd2d(-1.0, 1.0, 16).toarray(), 4000, 1e-8, True, True),
        ("pcg", "spd300", _spd(300, 21), 2000, 1e-10, True, False),
        ("gmres", "dh8", mg._dh(8).toarray(), 300, 1e-8, True, False),
        ("gmres", "nonsym200", _nonsym(200, 22), 300, 1e-10, True, True),
    ]
    index = []
    for kind, name, A, maxiter, tau, fom, jac in cases:
        assert isinstance(A, np.ndarray) and A.ndim == 2
        xex = np.random.default_rng(12345).random(A.shape[0])
        b = mg.ref_mvmult(A, xex)                      # np.dot(A, x_exact): the reference's dense mvmult
        res, hist = mg._run_ref(kind, A, b, maxiter, tau, fom, jac)
        orc = (mg.krylov.pcg if kind == "pcg" else mg.krylov.gmres)(
            A, b, maxiter=maxiter, tau=tau, fail_on_maxiter=fom, precond=mg._oracle_prec(A, jac))
        tag = "dense_%s_%s_%s" % (kind, name, mg._pname(jac))
        mg._check_same(tag, res, hist, orc)
        fname = tag + ".npz"
        np.savez_compressed(os.path.join(HERE, fname), A=A, b=b, x_exact=xex, hist=hist,
                            iters=np.int64(res.iters()), success=np.int64(bool(res.success())),
                            resid=np.float64(res.resid() if res.resid() is not None else np.nan),
                            soln=res.soln() if res.soln() is not None else np.zeros(0))
        sens = mg.sensitivity(kind, A, b, maxiter, tau, fom, jac, hist, res.soln())
        index.append(dict(file=fname, kind=kind, matrix=name, n=int(A.shape[0]), maxiter=maxiter, tau=tau,
                          fail_on_maxiter=fom, jacobi=mg._pname(jac) == "jacobi", precond=mg._pname(jac),
                          iters=int(res.iters()), success=bool(res.success()),
                          resid=None if res.resid() is None else float(res.resid()), sensitivity=sens))
        print("%-34s iters=%5d success=%s sens=%s" % (tag, res.iters(), res.success(), sens))
    import scipy
    with open(os.path.join(HERE, "manifest_dense.json"), "w") as f:
        json.dump(dict(cases=index, generator="tests/golden/make_dense.py", numpy=np.__version__,
                       scipy=scipy.__version__), f, indent=1)
    print("wrote", len(index), "dense fixtures")


if __name__ == "__main__":
    main()
