"""A/B of the AMG smoother's paired Gauss-Seidel sweeps (amg.hip gs_pair_kernel) on configs[4]'s workload:
-FD 8192^2, AMG(numIters=2, numLevels=5, nuPre=2, nuPost=2, Gauss-Seidel). Alternates pairing on / off
(psk_lab_amg_gs_pair) on the same hierarchy: AMG apply time (median of 5), PCG+AMG iterations per second
(6 iterations per solve, tau = 0), and whether the two applies agree bitwise. One JSON line on stdout.

    python tools/amg_pair_ab.py [--m 8192] [--rounds 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--no-lab", action="store_true",
                    help="pairing as built (on) only: for a PSK_LIBRARY build, which libpsk_lab.so must not be loaded beside")
    a = ap.parse_args()
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    lab = None if a.no_lab else N.load_lab()
    m, n = a.m, a.m * a.m
    t0 = time.time()
    A = -psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m).to_scipy()
    dA = psk.DeviceCSR.from_scipy(A)
    b = psk.Linear.spmv(dA, psk.DeviceVector.from_numpy(np.random.default_rng(12345).random(n)))
    M = psk.AMG(numIters=2, numLevels=5, smoother=psk.GaussSeidelSmoother).form(dA)
    del A
    print("setup %.1f s" % (time.time() - t0), file=sys.stderr, flush=True)

    def setp(v):
        if lab is None:
            return -1, -1
        on, el = ctypes.c_int32(), ctypes.c_int32()
        N.check(lab.psk_lab_amg_gs_pair(M.device_handle, v, ctypes.byref(on), ctypes.byref(el)), "gs_pair")
        return on.value, el.value

    v = psk.DeviceVector.from_numpy(np.random.default_rng(1).standard_normal(n))
    sol = psk.DeviceVector(n)

    def apply_ms(reps=5):
        M.apply(v)
        ts = []
        for _ in range(reps):
            N.check(N.lib.psk_synchronize(), "sync")
            t = time.perf_counter()
            M.apply(v)
            N.check(N.lib.psk_synchronize(), "sync")
            ts.append((time.perf_counter() - t) * 1e3)
        return float(np.median(ts))

    def pcg_its():
        ctl = N.PskCtl(maxiter=a.iters, tau=0.0, fail_on_maxiter=0, restart=0, check_every=0, time_kernels=0)
        res = N.PskResult()
        N.check(N.lib.psk_synchronize(), "sync")
        t = time.perf_counter()
        N.check(N.lib.psk_pcg(dA.handle, M.device_handle, b._p, sol._p, ctypes.byref(ctl), ctypes.byref(res), None,
                              N.PSK_DEVICE), "psk_pcg")
        N.check(N.lib.psk_synchronize(), "sync")
        return a.iters / (time.perf_counter() - t)

    out = {"workload": "-FDLaplacian2D %dx%d, AMG(numIters=2, numLevels=5, nu=2+2, GS)" % (m, m), "n": n}
    ys = {}
    res = {"on": {"apply_ms": [], "pcg_it_s": []}, "off": {"apply_ms": [], "pcg_it_s": []}}
    for r in range(a.rounds):
        for side, flag in ((("on", 1),) if lab is None else (("on", 1), ("off", 0))):
            on, el = setp(flag)
            out["levels_eligible"] = el
            res[side]["apply_ms"].append(apply_ms())
            res[side]["pcg_it_s"].append(pcg_its())
            if r == 0:
                y = M.apply(v).numpy()
                ys[side] = y
            print("round %d %s apply %.2f ms pcg %.2f it/s" % (r, side, res[side]["apply_ms"][-1],
                                                               res[side]["pcg_it_s"][-1]), file=sys.stderr, flush=True)
    setp(1)
    if "off" in ys:
        out["bitwise_equal"] = bool(np.array_equal(ys["on"], ys["off"]))
    else:
        res.pop("off")
    for side in res:
        out[side] = {"apply_ms_median": float(np.median(res[side]["apply_ms"])),
                     "pcg_it_s_median": float(np.median(res[side]["pcg_it_s"])), **res[side]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
