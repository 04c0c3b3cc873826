#!/usr/bin/env python3
"""Exit-fault probe (lab): one small solve of the chosen kind, then a normal interpreter exit. Run
under rocprofv3 to see which libpsk path leaves the process in a state whose exit() faults there.
    python tools/exit_probe.py pcg|ilu|amg|coop|lds|none

coop / lds: one 30000-row triangular solve on the sync-free schedule (a cooperative launch) / the LDS
schedule (a plain launch).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "pcg"
import pysolvers_amd as psk  # noqa: E402
from oracle import fdlap  # noqa: E402

A = fdlap.fd_laplacian_2d(-1.0, 1.0, 64)
b = A @ np.ones(A.shape[0])
ctl = psk.CommonSolverArgs(maxiter=20, tau=1e-8, showIters=False, showFinal=False)
if kind == "pcg":
    st = psk.PCG(control=ctl, precond=psk.Jacobi()).makeSolver().solve(A, b)
elif kind == "ilu":
    st = psk.GMRES(control=ctl, precond=psk.RightILUT(), restart=10).makeSolver().solve(A, b)
elif kind == "amg":
    st = psk.PCG(control=ctl, precond=psk.AMG(numIters=1, numLevels=2)).makeSolver().solve(-A, -b)
elif kind in ("coop", "lds"):
    import scipy.sparse as sp
    from pysolvers_amd.Linear import TriangularSolveChain
    n = 16000 if kind == "lds" else 30000
    L = (sp.diags(np.full(n, 2.0)) + sp.diags(np.full(n - 1, -0.5), -1)).tocsr()
    M = TriangularSolveChain(n, L=L)
    M.schedule("L", set="syncfree" if kind == "coop" else "lds")
    M.apply(np.ones(n))
    st = None
else:
    st = None
print(kind, None if st is None else (st.success(), st.iters()), flush=True)
