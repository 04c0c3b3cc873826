#!/usr/bin/env python3
"""RightILUT(FD m^2) apply time on the schedules the library picks (development probe, GPU): median
of 7 applies after one warm apply, plus a checksum of the result so builds / switches that must give
the same bits can be compared. Sync-free geometry experiments: PSK_SYNCFREE_PER_CU=k.

    python tools/sf_probe.py 2896
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def sched(N, h, f):
    import ctypes
    sc = ctypes.c_int32()
    N.check(N.lib.psk_prec_trisolve_schedule(h, f, -1, ctypes.byref(sc), None, None, None, None), "sched")
    return sc.value


def main():
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 2896
    t = time.time()
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    M = psk.RightILUT().form(dA)
    setup = time.time() - t
    v = psk.DeviceVector.from_numpy(np.random.default_rng(1).standard_normal(m * m))
    y = M.applyRight(v)
    ts = []
    for _ in range(7):
        N.check(N.lib.psk_synchronize(), "sync")
        t0 = time.perf_counter()
        y = M.applyRight(v)
        N.check(N.lib.psk_synchronize(), "sync")
        ts.append((time.perf_counter() - t0) * 1e3)
    out = {"m": m, "setup_s": setup, "per_cu": os.environ.get("PSK_SYNCFREE_PER_CU", "default"),
           "apply_ms": sorted(ts)[3], "all_ms": ts, "sha": hashlib.sha256(y.numpy().tobytes()).hexdigest()[:16],
           "schedules": [sched(N, M.device_handle, f) for f in (0, 1)]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
