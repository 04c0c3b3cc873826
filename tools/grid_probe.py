#!/usr/bin/env python3
"""Grid-schedule probe: the Gauss-Seidel factor triu(-FD m^2) solved with the grid schedule, timed,
and — with a library built with -DPSK_GRID_PROF — per-band s_memtime start / end, waits on the band
above and cycles spent waiting (development only; never part of the product path).

    PSK_LIBRARY=tools/bin/ab_prof/libpsk.so python tools/grid_probe.py --side 8192
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=8192)
    ap.add_argument("--level3", type=int, default=0, help="use the SA level-3 operator of -FD side^2 instead")
    args = ap.parse_args()
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear import TriangularSolveChain
    m = args.side
    A = -psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m).to_scipy()
    if args.level3:
        from pysolvers_amd.Linear import SmoothedAggregationMLHierarchy
        A = SmoothedAggregationMLHierarchy(A, numLevels=2).matrix(0).tocsr()
    U = sp.triu(A).tocsr()
    n = A.shape[0]
    M = TriangularSolveChain(n, U=U)
    out = {"side": m, "n": n, "level3": args.level3}
    v = psk.DeviceVector.from_numpy(np.random.default_rng(1).standard_normal(n))
    for sched in ("band", "grid"):
        M.schedule("U", set=sched)
        M.apply(v)
        N.check(N.lib.psk_synchronize(), "sync")
        t = time.perf_counter()
        for _ in range(3):
            M.apply(v)
        N.check(N.lib.psk_synchronize(), "sync")
        out[sched + "_ms"] = (time.perf_counter() - t) * 1e3 / 3
    if hasattr(N.lib, "psk_grid_prof_read"):
        nb = 8192
        buf = (ctypes.c_ulonglong * (8 * nb))()
        N.lib.psk_grid_prof_read(buf, nb)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
        used = a[:, 1] > 0
        a = a[used]
        t0 = a[:, 0].min()
        out["bands"] = int(len(a))
        out["probe"] = [{"band": int(b), "start": int(a[b, 0] - t0), "end": int(a[b, 1] - t0),
                         "dur": int(a[b, 1] - a[b, 0]), "waits": int(a[b, 2]), "wait_ticks": int(a[b, 3])}
                        for b in sorted(set([0, 1, 2, len(a) // 2, len(a) - 2, len(a) - 1]))]
        out["total_ticks"] = int(a[:, 1].max() - t0)
        out["bands_start_dur_waits_waitticks"] = [[int(a[b, 0] - t0), int(a[b, 1] - a[b, 0]), int(a[b, 2]), int(a[b, 3])]
                                                  for b in range(len(a))]
        out["waits_total"] = int(a[:, 2].sum())
        # per-step phases (s_memtime ticks summed over every step of every band; the last apply's)
        steps = 0.0 if args.level3 else float(m + 63) * len(a)   # FD: w = m, sigma = 1: S = w + 63 per band
        ph = {"records_rhs_ready": a[:, 4].sum(), "lds_ring_reads": a[:, 5].sum(), "fma_div": a[:, 6].sum(),
              "ring_write_store_issue": a[:, 7].sum(), "ext_wait": a[:, 3].sum()}
        tot = float(sum(ph.values()))
        out["phase_share"] = {k: float(v) / tot for k, v in ph.items()}
        out["phase_ticks_total"] = {k: int(v) for k, v in ph.items()}
        if steps:
            out["ticks_per_step"] = {k: float(v) / steps for k, v in ph.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
