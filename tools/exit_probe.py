#!/usr/bin/env python3
"""Exit-fault probe (lab): one small solve of the chosen kind, then a normal interpreter exit. Run
under rocprofv3 to see which libpsk path leaves the process in a state whose exit() faults there.
    python tools/exit_probe.py pcg|ilu|amg|none
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
else:
    st = None
print(kind, None if st is None else (st.success(), st.iters()), flush=True)
