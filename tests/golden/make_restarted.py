#!/usr/bin/env python3
"""Golden fixtures for restarted GMRES(m), pinned to the REFERENCE's own GMRES solve.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_restarted.py

The reference has no restart (GMRESSolver.py:104: one Krylov space of dimension maxiter; it crashes
with NameError at :180 when maxiter is reached). GMRES(m) here is cycles of the reference's loop on
the residual system A dx = r_c (oracle/krylov.py gmres_restarted). This script checks every cycle of
the oracle against the reference itself, bit for bit:

* cycle c's rhs r_c (r_0 = b, r_c = b - mvmult(A, x_c)) is handed to the reference's
  GMRESSolver.solve (patched only for its missing `precond` attribute, GMRESSolver.py:71) with a
  tau that makes the reference stop exactly after the cycle's number of steps: for a full cycle,
  the last recursive residual of the cycle over ||r_c|| (times 1 + 1e-12); for the converging
  cycle, tau * ||b|| / ||r_c||;
* the reference's per-step residuals (reportIter) must equal the oracle cycle's, its step count the
  cycle's, and its returned x the oracle cycle's dx, all bitwise.

Fixtures (data only) go to tests/golden/gmres_restart*.npz + manifest_restarted.json.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.dont_write_bytecode = True

import make_golden as mg                                  # noqa: E402  (installs the stand-ins, imports the reference)
from oracle import fdlap, krylov                          # noqa: E402

CASES = [
    # (matrix name, builder, restart, maxiter, tau, fail_on_maxiter, precond)
    ("fd32", lambda: mg.ref_fd2d(-1.0, 1.0, 32), 30, 600, 1e-8, True, "jacobi"),
    ("fd64", lambda: mg.ref_fd2d(-1.0, 1.0, 64), 30, 2000, 1e-8, True, "jacobi"),
    ("fd64", lambda: mg.ref_fd2d(-1.0, 1.0, 64), 30, 200, 1e-8, True, "ilut"),
    ("fd128", lambda: mg.ref_fd2d(-1.0, 1.0, 128), 30, 200, 1e-8, True, "ilut"),
    ("dh10", lambda: mg._dh(10), 30, 1000, 1e-8, True, "identity"),
    ("dh10", lambda: mg._dh(10), 30, 300, 1e-8, True, "ilut"),
    ("dh8", lambda: mg._dh(8), 10, 400, 1e-8, True, "identity"),
    # maxiter reached mid-cycle (fail and no-fail): handleMaxiter(maxiter - 1, ...)
    ("fd32_maxiter45_fail", lambda: mg.ref_fd2d(-1.0, 1.0, 32), 30, 45, 1e-8, True, "jacobi"),
    ("fd32_maxiter45_nofail", lambda: mg.ref_fd2d(-1.0, 1.0, 32), 30, 45, 1e-8, False, "jacobi"),
]


def ref_cycle(A, r, steps, tau_ref, jac):
    """The reference's GMRES solve on (A, r) with maxiter large enough never to reach :180."""
    res, hist = mg._run_ref("gmres", A, r, steps + 50, tau_ref, True, jac)
    return res, hist


def main():
    index = []
    for name, build, restart, maxiter, tau, fom, jac in CASES:
        A = build()
        b, xex = fdlap.manufactured_rhs(A, 12345)
        cyc = []
        prec = mg._oracle_prec(A, jac)
        orc = krylov.gmres_restarted(A, b, restart, maxiter=maxiter, tau=tau, fail_on_maxiter=fom, precond=prec,
                                     cycles=cyc)
        norm_b = np.linalg.norm(b)
        pos = 0
        for c, (r, steps, dx) in enumerate(cyc):
            h_orc = orc["hist"][pos:pos + steps]
            nr = np.linalg.norm(r)
            if h_orc[-1] <= tau * norm_b or len(h_orc) < min(restart, maxiter - pos):
                tau_ref = tau * norm_b / nr                          # the cycle converged (or broke down)
            else:
                tau_ref = h_orc[-1] / nr * (1.0 + 1e-12)             # a full cycle: stop after its last step
            res, h_ref = ref_cycle(A, r, steps, tau_ref, jac)
            tag = "%s cycle %d" % (name, c)
            assert res.iters() == steps, (tag, res.iters(), steps)
            assert np.array_equal(h_ref, h_orc), tag
            assert np.array_equal(res.soln(), dx), tag
            pos += steps
        assert pos == len(orc["hist"])
        tag = "gmres_restart%d_%s_%s" % (restart, name, jac)
        payload = dict(b=b, x_exact=xex, hist=orc["hist"], maxiter=np.int64(maxiter), tau=np.float64(tau),
                       fail_on_maxiter=np.int64(fom), restart=np.int64(restart), precond=np.array(jac),
                       iters=np.int64(orc["iters"]), success=np.int64(bool(orc["success"])),
                       resid=np.float64(orc["resid"]), soln=orc["soln"], **mg._csr_arrays(A))
        np.savez_compressed(os.path.join(HERE, tag + ".npz"), **payload)
        index.append(dict(file=tag + ".npz", kind="gmres", matrix=name, n=int(A.shape[0]), nnz=int(A.nnz),
                          restart=restart, maxiter=maxiter, tau=tau, fail_on_maxiter=fom, precond=jac,
                          iters=int(orc["iters"]), success=bool(orc["success"]), resid=float(orc["resid"]),
                          cycles=len(cyc), msg=orc["msg"]))
        print("%-44s iters=%4d cycles=%3d success=%s (every cycle == reference)" % (
            tag, orc["iters"], len(cyc), orc["success"]))
    with open(os.path.join(HERE, "manifest_restarted.json"), "w") as f:
        json.dump({"cases": index, "generator": "tests/golden/make_restarted.py", "numpy": np.__version__}, f,
                  indent=1)


if __name__ == "__main__":
    main()
