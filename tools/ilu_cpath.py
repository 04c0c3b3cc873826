#!/usr/bin/env python3
"""Critical-path model of the ILUT triangular solves (host only, lab tool).

    python tools/ilu_cpath.py 2896 [--P 256] [--W 16]

For the reference's ILUT factors of FD m^2 (spilu(drop_tol=1e-3, fill_factor=15), ILUTPreconditioner.py:51-53;
cached by tools/ilu_dag.py) and each factor:
  1. the dependency levels and the share of TIGHT edges (parent one level below its child: the edges every
     longest path is made of) that cross CUs under the current sync-free deal (solve position k, in level
     order, to enrolled wave k mod W_e; workgroups of 4 waves dealt round-robin to the CUs);
  2. the makespan of a partitioned schedule (one workgroup of --W waves per CU, rows of a part run in level
     order, each on its part's earliest-free wave) for two DAG-aware partitions:
       tiles  - T x T tiles of the grid point each factor row belongs to (the mesh's own locality),
       strips - the round-2 partitioned schedule's strips of the natural index (the calibration case),
       level  - each level cut into P contiguous chunks of its rows in grid-point order (consecutive
                levels' chunks line up along the wavefront, so tight edges mostly stay in their chunk);
     priced at the measured hand-offs: a dependency inside a CU costs `a`, across CUs `b`, every row `c`
     of its wave's time. Two readings of the measured prices (profiles/r4_part_handoff_phases.txt: the
     LDS hand-off 0.53 us; sync-free 1.09 us per level all-in, of which the cross-CU hop ~0.88):
       all-in  a + c = 0.53, b + c = 1.09 (c = 0.21)
       hop     a = 0.53, b = 0.88, c = 0.21
Prints one JSON object; the verdict's bar is a projected apply (L + U) <= 20 ms.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ilu_dag import factors, simulate, strict, weighted_path  # noqa: E402


def tight_cross_share(S, lev, W_e, P):
    """share of tight edges whose endpoints sit on different CUs under the sync-free deal"""
    n = S.shape[0]
    order = np.lexsort((np.arange(n), lev))
    pos = np.empty(n, np.int64)
    pos[order] = np.arange(n)
    wave = pos % W_e
    cu = (wave // 4) % P
    rows = np.repeat(np.arange(n), np.diff(S.indptr))
    par = S.indices
    tight = lev[par] == lev[rows] - 1
    cross = cu[par[tight]] != cu[rows[tight]]
    return float(tight.mean()), float(cross.mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("m", type=int)
    ap.add_argument("--P", type=int, default=256)
    ap.add_argument("--W", type=int, default=16)
    ap.add_argument("--We", type=int, default=7168, help="enrolled sync-free waves (7 workgroups x 4 waves x 256 CUs)")
    a_ = ap.parse_args()
    m, P, W = a_.m, a_.P, a_.W
    L, U, pr, pc = factors(m)
    n = m * m
    Ls, Us = strict(L, True), strict(U, False)
    ptL = np.empty(n, np.int64)
    ptL[pr] = np.arange(n)
    ptU = np.empty(n, np.int64)
    ptU[pc] = np.arange(n)
    prices = {"all-in": (0.32, 1.09 - 0.21, 0.21), "hop": (0.53, 0.88, 0.21)}
    out = {"m": m, "P": P, "W": W, "prices_us": {k: dict(a=v[0], b=v[1], c=v[2]) for k, v in prices.items()},
           "factors": {}}
    tot = {}
    for name, S, lower, pt in (("L", Ls, True, ptL), ("U", Us, False, ptU)):
        _, lev = weighted_path(S, lower, np.zeros(n, np.int32), 1.0, 1.0, 0.0)
        nl = int(lev.max()) + 1
        tshare, cross = tight_cross_share(S, lev, a_.We, P)
        f = {"levels": nl, "rows_per_level": n / nl, "entries_per_row": S.nnz / n,
             "tight_edge_share": tshare, "syncfree_tight_cross_cu": cross, "model_ms": {}}
        # partitions
        T = int(round(m / np.sqrt(P)))
        gx, gy = pt % m, pt // m
        nt = (m + T - 1) // T
        tiles = ((gy // T) * nt + gx // T) % P
        # level chunks: rows of each level sorted by grid point, cut into P contiguous chunks
        order = np.lexsort((pt, lev))
        cnt = np.bincount(lev, minlength=nl)
        start = np.concatenate(([0], np.cumsum(cnt)[:-1]))
        q = np.empty(n, np.int64)
        q[order] = np.arange(n) - np.repeat(start, cnt)
        chunks = (q * P) // np.maximum(cnt[lev], 1)
        rows = np.repeat(np.arange(n), np.diff(S.indptr))
        par = S.indices
        tight = lev[par] == lev[rows] - 1
        strips = (pt * P) // n   # the round-2 partitioned schedule's strips of the natural index (calibration:
        #                          measured 31.4 ms vs sync-free 27.1 at 2896^2, profiles/r3_part_forced.txt)
        for pname, wg in (("strips", strips), ("tiles", tiles), ("level", chunks)):
            wg = wg.astype(np.int32)
            f["tight_cross_" + pname] = float((wg[par[tight]] != wg[rows[tight]]).mean())
            for k, (a, b, c) in prices.items():
                ms = simulate(S, lev, wg, W, a, b, c, dyn=True) / 1e3
                f["model_ms"]["%s/%s" % (pname, k)] = ms
                tot["%s/%s" % (pname, k)] = tot.get("%s/%s" % (pname, k), 0.0) + ms
        for k, (a, b, c) in prices.items():
            sf = nl * (b + c) / 1e3
            f["model_ms"]["syncfree/%s" % k] = sf
            tot["syncfree/%s" % k] = tot.get("syncfree/%s" % k, 0.0) + sf
            f["model_ms"]["all_in_cu_bound/%s" % k] = nl * (a + c) / 1e3
        out["factors"][name] = f
        print(json.dumps({name: f}), flush=True)
    out["apply_ms"] = tot
    out["best_partitioned_ms"] = min(v for k, v in tot.items() if not k.startswith("syncfree"))
    out["builds"] = out["best_partitioned_ms"] <= 20.0
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
