#!/usr/bin/env python3
"""configs[4]: PCG + AMG V-cycle preconditioner on -FDLaplacian2D(m), one GPU — PCG iterations/s.

    python tools/bench_amg.py --side 8192 --levels 5 --iters 10 [--smoother gs|jacobi] [--cycles 2]

-A is the sign FDBratu2D.py:15 uses (A = -FDLaplacian2D is SPD). The hierarchy is built on the
host (O(nnz) SA setup, timed separately); the timed region is ONE PCG solve of exactly `iters`
iterations (tau = 0, failOnMaxiter = False; PCG+AMG does not converge on this matrix, SURVEY.md §6,
so iterations/s is the protocol), operands resident in HBM. Also reports one AMG apply and one
fine-level Gauss-Seidel sweep (triu(A)^-1) alone.

numLevels: the reference's default (2) leaves a coarse level of ~n/6 unknowns that its per-call
SuperLU factorisation cannot handle at this size (SuperLU fails at FD 4096^2 already, see
tools/bench_gmres.py); 5 levels leave a ~10^5-unknown coarse problem at m = 8192.
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
    ap.add_argument("--levels", type=int, default=5)
    ap.add_argument("--cycles", type=int, default=2)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--smoother", default="gs", choices=["gs", "jacobi"])
    ap.add_argument("--coarse", default="auto", choices=["auto", "dense", "lu"])
    args = ap.parse_args()
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N

    m = args.side
    n = m * m
    t = time.time()
    A = -psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m).to_scipy()
    dA = psk.DeviceCSR.from_scipy(A)
    x = psk.DeviceVector.from_numpy(np.random.default_rng(12345).random(n))
    b = psk.Linear.spmv(dA, x)
    del x
    out = dict(side=m, n=n, levels=args.levels, cycles=args.cycles, smoother=args.smoother, iters=args.iters)
    t1 = time.time()
    sm = psk.JacobiSmoother if args.smoother == "jacobi" else psk.GaussSeidelSmoother
    M = psk.AMG(numIters=args.cycles, numLevels=args.levels, smoother=sm, coarse=args.coarse).form(dA)
    del A
    out["amg_setup_s"] = time.time() - t1
    out["level_sizes"] = M.levels()
    if args.smoother == "gs":
        info = M._S[-1].operator.device_info()
        out["fine_gs_levels"] = info["levels_u"]
    v = psk.DeviceVector.from_numpy(np.random.default_rng(1).standard_normal(n))
    M.apply(v)
    N.check(N.lib.psk_synchronize(), "sync")
    reps = 3
    t2 = time.perf_counter()
    for _ in range(reps):
        M.apply(v)
    N.check(N.lib.psk_synchronize(), "sync")
    out["amg_apply_ms"] = (time.perf_counter() - t2) * 1e3 / reps
    if args.smoother == "gs":
        S = M._S[-1].operator
        info = S.schedule("U")
        out["fine_gs_schedule"] = info
        chosen = info["schedule"]
        for sched in ("syncfree", "band", "grid"):
            try:
                S.schedule("U", set=sched)
            except N.PskError:
                continue
            S.apply(v)
            N.check(N.lib.psk_synchronize(), "sync")
            t3 = time.perf_counter()
            for _ in range(reps):
                S.apply(v)
            N.check(N.lib.psk_synchronize(), "sync")
            out["fine_gs_sweep_ms_" + sched] = (time.perf_counter() - t3) * 1e3 / reps
        S.schedule("U", set=chosen)
        out["coarse_levels_schedules"] = [M._S[k].operator.schedule("U")["schedule"] for k in range(1, args.levels)]

    def timed(op, vec, reps=3):
        op.apply(vec)
        N.check(N.lib.psk_synchronize(), "sync")
        t4 = time.perf_counter()
        for _ in range(reps):
            op.apply(vec)
        N.check(N.lib.psk_synchronize(), "sync")
        return (time.perf_counter() - t4) * 1e3 / reps

    # per level: smoother sweep operator (S^-1) time and schedule; coarse solve time
    per = []
    for k in range(1, args.levels):
        op = M._S[k].operator
        vk = psk.DeviceVector.from_numpy(np.random.default_rng(k).standard_normal(M.levels()[k]))
        e = dict(level=k, n=M.levels()[k], op_ms=timed(op, vk))
        if args.smoother == "gs":
            e.update(op.schedule("U"), dep_levels=op.device_info()["levels_u"])
            chosen = e["schedule"]
            for sched in ("syncfree", "band", "grid", "part"):
                try:
                    op.schedule("U", set=sched)
                except N.PskError:
                    continue
                e["op_ms_" + sched] = timed(op, vk)
            op.schedule("U", set=chosen)
        per.append(e)
    v0 = psk.DeviceVector.from_numpy(np.random.default_rng(0).standard_normal(M.levels()[0]))
    co = M._coarse
    if M.coarse_kind == "dense":
        n0 = M.levels()[0]
        ms = timed(co, v0)
        per.append(dict(level=0, n=n0, coarse="dense", coarse_solve_ms=ms,
                        gemv_gb_s=n0 * ((n0 + 7) // 8 * 8) * 8 / (ms * 1e-3) / 1e9))
    else:
        per.append(dict(level=0, n=M.levels()[0], coarse="lu", coarse_solve_ms=timed(co, v0), L=co.schedule("L"),
                        U=co.schedule("U"), dep_levels=[co.device_info()["levels_l"], co.device_info()["levels_u"]],
                        nnz=[co.device_info()["nnz_l"], co.device_info()["nnz_u"]]))
    if M.coarse_kind == "lu" and M.levels()[0] <= 18432:   # coarse solve under each schedule it can run, then back to the chosen one
        chosen = (co.schedule("L")["schedule"], co.schedule("U")["schedule"])
        for sched in ("syncfree", "lds"):
            co.schedule("L", set=sched)
            co.schedule("U", set=sched)
            per[-1]["coarse_solve_ms_" + sched] = timed(co, v0)
        co.schedule("L", set=chosen[0])
        co.schedule("U", set=chosen[1])
    out["per_level"] = per
    out["setup_s"] = time.time() - t
    sol = psk.DeviceVector(n)

    def run(k):
        ctl = N.PskCtl(maxiter=k, tau=0.0, fail_on_maxiter=0, restart=0, check_every=0, time_kernels=0)
        res = N.PskResult()
        N.check(N.lib.psk_pcg(dA.handle, M.device_handle, b._p, sol._p, ctypes.byref(ctl), ctypes.byref(res), None,
                              N.PSK_DEVICE), "psk_pcg")
        return res

    run(1)
    N.check(N.lib.psk_synchronize(), "sync")
    t0 = time.perf_counter()
    res = run(args.iters)
    N.check(N.lib.psk_synchronize(), "sync")
    dt = time.perf_counter() - t0
    out.update(pcg_it_per_s=args.iters / dt, ms_per_it=dt * 1e3 / args.iters, status=int(res.status),
               iters_done=int(res.iters), rec_resid_ratio=res.resid_recursive / res.norm_b)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
