#!/usr/bin/env python3
"""configs[2]: GMRES(restart) + right ILUT on FDLaplacian2D m x m, one GPU — Arnoldi steps/s.

    python tools/bench_gmres.py --side 4096 --restart 30 --steps 60 [--precond ilut|jacobi|identity]

The matrix is built on the device (DeviceCSR.fd_laplacian_2d); for ILUT it is downloaded once
and factored on the host by scipy SuperLU with the reference's arguments (setup, timed
separately); the timed region is ONE GMRES solve of exactly `steps` Arnoldi steps (tau = 0,
failOnMaxiter = False), operands resident in HBM. Also reports the ILU apply time alone and the
reference-path cost of one ILU.solve on the host for scale.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=1024)
    ap.add_argument("--restart", type=int, default=30)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--precond", default="ilut", choices=["ilut", "jacobi", "identity"])
    args = ap.parse_args()
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N

    m = args.side
    n = m * m
    t = time.time()
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    x = psk.DeviceVector.from_numpy(np.random.default_rng(12345).random(n))
    b = psk.Linear.spmv(dA, x)
    del x
    out = {"side": m, "n": n, "restart": args.restart, "steps": args.steps, "precond": args.precond}
    M = None
    if args.precond == "ilut":
        t1 = time.time()
        try:
            M = psk.RightILUT().form(dA)
        except RuntimeError as e:
            # scipy 1.15.3 SuperLU cannot form the reference's ILUT (drop_tol=1e-3, fill_factor=15)
            # at FD 4096^2: SUPERLU_MALLOC fails in intCalloc after ~7 s, on this container too.
            out.update(error="reference ILUT factorization failed: %s" % e, ilut_setup_s=time.time() - t1)
            print(json.dumps(out), flush=True)
            sys.exit(3)
        out["ilut_setup_s"] = time.time() - t1
        out["ilu_nnz_L"], out["ilu_nnz_U"] = int(M.ILU().L.nnz), int(M.ILU().U.nnz)
        v = psk.DeviceVector.from_numpy(np.random.default_rng(1).standard_normal(n))
        M.applyRight(v)
        reps = 5
        N.check(N.lib.psk_synchronize(), "sync")
        t2 = time.perf_counter()
        for _ in range(reps):
            w = M.applyRight(v)
        N.check(N.lib.psk_synchronize(), "sync")
        out["ilu_apply_ms"] = (time.perf_counter() - t2) * 1e3 / reps
        vh = v.numpy()
        t3 = time.perf_counter()
        M.ILU().solve(vh)
        out["host_superlu_solve_ms"] = (time.perf_counter() - t3) * 1e3
        pt_h, kind = M.device_handle, None
    elif args.precond == "jacobi":
        M = psk.JacobiPreconditionerType().form(dA)
        pt_h = M.device_handle
    else:
        pt_h = None
    out["setup_s"] = time.time() - t
    sol = psk.DeviceVector(n)

    def run(steps):
        ctl = N.PskCtl(maxiter=steps, tau=0.0, fail_on_maxiter=0, restart=args.restart, check_every=0,
                       time_kernels=0)
        res = N.PskResult()
        N.check(N.lib.psk_gmres(dA.handle, pt_h, b._p, sol._p, ctypes.byref(ctl), ctypes.byref(res), None,
                                N.PSK_DEVICE), "psk_gmres")
        return res

    run(min(args.restart, args.steps))     # warm-up cycle
    N.check(N.lib.psk_synchronize(), "sync")
    t0 = time.perf_counter()
    res = run(args.steps)
    N.check(N.lib.psk_synchronize(), "sync")
    dt = time.perf_counter() - t0
    out.update(steps_per_s=args.steps / dt, ms_per_step=dt * 1e3 / args.steps, status=int(res.status),
               rec_resid_ratio=res.resid_recursive / res.norm_b)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
