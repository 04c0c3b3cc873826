#!/usr/bin/env python3
"""Development probe: per-phase cycles of one band block's local levels (libpsk built with
-DPSK_BAND_PROF into tools/bin/prof/, loaded through PSK_LIBRARY).

    PSK_LIBRARY=tools/bin/prof/libpsk.so python tools/band_prof.py --side 8192
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=8192)
    args = ap.parse_args()
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear import TriangularSolveChain
    m = args.side
    A = -psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m).to_scipy()
    U = sp.triu(A).tocsr()
    M = TriangularSolveChain(U.shape[0], U=U)
    M.schedule("U", set="band")
    v = psk.DeviceVector.from_numpy(np.random.default_rng(0).standard_normal(U.shape[0]))
    M.apply(v)
    N.check(N.lib.psk_synchronize(), "sync")
    buf = (ctypes.c_ulonglong * 8)()
    assert N.lib.psk_band_prof_read(buf) == 0
    lv = buf[4]
    print(json.dumps({"side": m, "levels": lv, "info": M.schedule("U"),
                      "per_level": {"phase0": buf[0] / lv, "phase1": buf[1] / lv, "phase2": buf[2] / lv,
                                    "slot3": buf[3] / lv},
                      "phases": "band: control+advance, record+ring reads, sum+div+store, waitcnt+barrier (cycles); "
                                "narrow: control+chunk wait, record+ring reads, sum+div+store+waitcnt (cycles), "
                                "sentinel snapshots met per level"}))


if __name__ == "__main__":
    main()
