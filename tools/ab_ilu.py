#!/usr/bin/env python3
"""ILU apply time per triangular-solve schedule (lab tool): RightILUT of FD m^2 (the reference's
spilu call) formed with PSK_TRISOLVE_STRIP=1 (both layouts built), then the apply timed with each
factor on the strip, sync-free and (where the model planned it) the chosen schedule; max relative
deviation from SuperLU's ILU.solve. One JSON line per side.

    PSK_TRISOLVE_VERBOSE=1 python tools/ab_ilu.py 1024 2896
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    os.environ["PSK_TRISOLVE_STRIP"] = "1"
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    from oracle import fdlap
    names = {0: "syncfree", 1: "band", 2: "lds", 3: "grid", 4: "part", 5: "strip"}
    for m in [int(a) for a in sys.argv[1:]] or [1024]:
        A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
        t0 = time.time()
        M = psk.RightILUT().form(A)
        setup = time.time() - t0
        h = M.device_handle
        info = M.device_info()
        v = np.random.default_rng(1).standard_normal(m * m)
        dv = psk.DeviceVector.from_numpy(v)
        ref = M.ILU().solve(v)

        def sched(which, s=-1):
            sc = ctypes.c_int32()
            N.check(N.lib.psk_prec_trisolve_schedule(h, which, s, ctypes.byref(sc), None, None, None, None), "sched")
            return names[sc.value]

        def timed():
            M.applyRight(dv)
            ts = []
            for _ in range(5):
                N.check(N.lib.psk_synchronize(), "sync")
                t = time.perf_counter()
                M.applyRight(dv)
                N.check(N.lib.psk_synchronize(), "sync")
                ts.append((time.perf_counter() - t) * 1e3)
            out = M.applyRight(v)
            return sorted(ts)[2], float(np.linalg.norm(out - ref) / np.linalg.norm(ref))
        res = {"m": m, "n": m * m, "setup_s": setup, "levels_l": info["levels_l"], "levels_u": info["levels_u"]}
        for lo, up in (("strip", "strip"), ("syncfree", "syncfree"), ("strip", "syncfree"), ("syncfree", "strip")):
            sched(0, 5 if lo == "strip" else 0)
            sched(1, 5 if up == "strip" else 0)
            ms, dev = timed()
            res["%s+%s" % (lo, up)] = {"apply_ms": ms, "rel_dev_vs_superlu": dev}
        print(json.dumps(res), flush=True)
        del M, dv


if __name__ == "__main__":
    main()
