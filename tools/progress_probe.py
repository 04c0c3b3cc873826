#!/usr/bin/env python3
"""Lab probe of the triangular solves beside occupiers (tests/test_gpu_progress.py's setting, verbose).

    python tools/progress_probe.py [--m 384] [--wgs 128[,192,...]] [--lds 102400] [--seconds 8] [--sched syncfree]
                                   [--factor ilu|gs]

--factor gs: the Gauss-Seidel factor triu(-FD m^2) as a one-factor chain (schedules band / grid / syncfree).

Prints, for an idle device and then beside `wgs` occupier workgroups: the apply's wall time, the
enrolled workers / grid of each sync-free factor, whether the occupiers timed out, the error word, and
whether the result kept its bits.
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
    ap.add_argument("--m", type=int, default=384)
    ap.add_argument("--wgs", default="128")
    ap.add_argument("--factor", default="ilu", choices=["ilu", "gs"])
    ap.add_argument("--dispatch", default="", help="NWG,LDS_BYTES,USEC: the dispatch probe kernel instead of a solve")
    ap.add_argument("--lds", type=int, default=100 * 1024)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--sched", default="syncfree")
    a = ap.parse_args()
    os.environ.setdefault("PSK_NO_TORCH", "1")
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    if a.dispatch:
        nwg, lds, us = (float(v) for v in a.dispatch.split(","))
        nwg, lds = int(nwg), int(lds)
        for wgs in [0] + [int(w) for w in a.wgs.split(",")]:
            if wgs:
                N.check(N.load_lab().psk_lab_occupy_begin(wgs, a.lds, a.seconds), "occupy_begin")
            rec = np.zeros(3 * nwg, np.int64)
            t0 = time.perf_counter()
            N.check(N.load_lab().psk_lab_dispatch_probe(nwg, lds, us, N.ptr(rec)), "dispatch_probe")
            ms = (time.perf_counter() - t0) * 1e3
            to = N.I32()
            if wgs:
                N.check(N.load_lab().psk_lab_occupy_end(ctypes.byref(to)), "occupy_end")
            r = rec.reshape(nwg, 3)
            st = (r[:, 0] - r[:, 0].min()) / 100.0   # us
            print(json.dumps({"phase": "dispatch", "wgs": wgs, "nwg": nwg, "lds": lds, "usec": us, "ms": ms,
                              "timed_out": to.value, "start_us_quantiles": [float(np.quantile(st, q)) for q in (0, .25, .5, .75, 1)],
                              "per_xcd": np.bincount(r[:, 2], minlength=8).tolist()}), flush=True)
        return
    from oracle import fdlap
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, a.m)
    code = {"syncfree": 0, "band": 1, "lds": 2, "grid": 3, "part": 4}[a.sched]
    if a.factor == "gs":
        import scipy.sparse as sp
        from pysolvers_amd.Linear import TriangularSolveChain
        M = TriangularSolveChain(A.shape[0], U=sp.triu(-A).tocsr())
        facs = (1,)
    else:
        M = psk.RightILUT().form(psk.DeviceCSR.from_scipy(A))
        facs = (0, 1)
    for f in facs:
        N.check(N.lib.psk_prec_trisolve_schedule(M.device_handle, f, code, None, None, None, None, None), "schedule")
    v = psk.DeviceVector.from_numpy(np.random.default_rng(5).standard_normal(A.shape[0]))

    def workers():
        out = []
        for f in facs:
            e, g = N.I32(), N.I32()
            N.check(N.load_lab().psk_lab_trisolve_workers(M.device_handle, f, ctypes.byref(e), ctypes.byref(g)), "workers")
            out.append((e.value, g.value))
        return out

    out = psk.DeviceVector(A.shape[0])

    def timed():   # nothing allocated or freed inside (hipFree waits for the whole device)
        t0 = time.perf_counter()
        try:
            N.check(N.lib.psk_prec_apply(M.device_handle, A.shape[0], v._p, out._p, N.PSK_DEVICE), "apply")
            err = None
        except N.PskError as e:
            err = str(e)
        return (time.perf_counter() - t0) * 1e3, err

    ms, err = timed()
    print(json.dumps({"phase": "idle", "ms": ms, "err": err, "workers": workers()}), flush=True)
    ms, err = timed()
    ref = out.numpy()
    print(json.dumps({"phase": "idle2", "ms": ms, "err": err, "workers": workers()}), flush=True)
    for wgs in (int(w) for w in a.wgs.split(",")):
        N.check(N.load_lab().psk_lab_occupy_begin(wgs, a.lds, a.seconds), "occupy_begin")
        ms, err = timed()
        to = N.I32()
        N.check(N.load_lab().psk_lab_occupy_end(ctypes.byref(to)), "occupy_end")
        xcc = (N.I32 * 8)()
        N.check(N.load_lab().psk_lab_occupy_xcc(xcc), "occupy_xcc")
        y = out.numpy()
        rec = {"phase": "occupied", "wgs": wgs, "xcc": list(xcc), "ms": ms, "err": err, "timed_out": to.value,
               "workers": workers(),
               "same_bits": None if y is None else bool(np.array_equal(y.view(np.uint64), ref.view(np.uint64)))}
        if a.sched == "grid" and hasattr(N.lib, "psk_grid_prof_read"):   # a -DPSK_GRID_PROF lab build
            nb = (a.m + 63) // 64
            buf = (ctypes.c_ulonglong * (8 * nb))()
            N.lib.psk_grid_prof_read(buf, nb)
            b = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
            t0 = b[:, 6].min()
            rec["bands"] = [{"band": i, "xcd": int(b[i, 4]), "wg": int(b[i, 5]), "start_us": (b[i, 6] - t0) / 100.0,
                             "end_us": (b[i, 7] - t0) / 100.0} for i in range(nb)]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
