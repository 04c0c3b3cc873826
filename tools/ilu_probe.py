#!/usr/bin/env python3
"""ILUT apply timing per triangular-solve schedule (development probe, GPU).

    python tools/ilu_probe.py M [M ...]

Forms RightILUT(FD m^2) with the partitioned layout built (PSK_TRISOLVE_PART=1), then times the
apply with both factors on the partitioned and on the sync-free schedule (median of 5), checks the
two bit for bit, and prints the host cost-model estimates. One JSON line per m.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    for m in [int(a) for a in sys.argv[1:]] or [1024]:
        t = time.time()
        dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
        os.environ["PSK_TRISOLVE_PART"] = "1"
        os.environ["PSK_TRISOLVE_VERBOSE"] = "1"
        M = psk.RightILUT().form(dA)
        del os.environ["PSK_TRISOLVE_PART"]
        setup = time.time() - t
        h = M.device_handle
        n = m * m
        v = psk.DeviceVector.from_numpy(np.random.default_rng(1).standard_normal(n))
        out = {"m": m, "setup_s": setup}
        info = M.device_info()
        out.update(levels_l=info["levels_l"], levels_u=info["levels_u"], nnz_l=info["nnz_l"], nnz_u=info["nnz_u"])
        res = {}
        for sched, code in (("part", 4), ("syncfree", 0)):
            for f in (0, 1):
                sc, e1, e2 = ctypes.c_int32(), ctypes.c_double(), ctypes.c_double()
                N.check(N.lib.psk_prec_trisolve_schedule(h, f, code, ctypes.byref(sc), None, None, ctypes.byref(e1),
                                                         ctypes.byref(e2)), "sched")
            M.applyRight(v)
            ts = []
            for _ in range(5):
                N.check(N.lib.psk_synchronize(), "sync")
                t0 = time.perf_counter()
                y = M.applyRight(v)
                N.check(N.lib.psk_synchronize(), "sync")
                ts.append((time.perf_counter() - t0) * 1e3)
            res[sched] = y.numpy()
            out[sched + "_ms"] = sorted(ts)[2]
            out[sched + "_all_ms"] = ts
        out["bit_identical"] = bool(np.array_equal(res["part"], res["syncfree"]))
        if hasattr(N.lib, "psk_part_prof_read"):   # a -DPSK_PART_PROF build (scripts/build_variant.sh)
            buf = (ctypes.c_ulonglong * 8)()
            for f in (0, 1):
                for g in (0, 1):
                    N.check(N.lib.psk_prec_trisolve_schedule(h, g, 4 if g == f else 0, None, None, None, None, None),
                            "sched")
                M.applyRight(v)
                N.check(N.lib.psk_synchronize(), "sync")
                N.lib.psk_part_prof_read(buf)
                M.applyRight(v)
                N.check(N.lib.psk_synchronize(), "sync")
                N.lib.psk_part_prof_read(buf)
                c = list(buf)
                waves = 256 * 16
                out["prof_" + "LU"[f]] = {
                    "wave_cycles_mean": c[0] / waves, "local_wait_mean": c[1] / waves, "remote_wait_mean": c[2] / waves,
                    "rows": c[3], "local_waits": c[4], "remote_waits": c[5], "slot_reuses": c[6],
                    "wave_cycles_max": c[7]}
        out["us_per_level_part"] = out["part_ms"] * 1e3 / (info["levels_l"] + info["levels_u"])
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
