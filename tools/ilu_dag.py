#!/usr/bin/env python3
"""Dependency-DAG analysis of the ILUT factors (development tool, host only).

    python tools/ilu_dag.py M [T ...]

Factors FD m^2 with the reference's spilu call (ILUTPreconditioner.py:51-53), maps every factor row
to its grid point (L row perm_r[i] <-> equation i, U row perm_c[j] <-> unknown j) and reports, for
2-D tilings of the grid into T x T tiles, the critical path of the solve when a dependency inside a
tile costs `a` and one across tiles costs `b` (us): the latency a tile-partitioned schedule could
reach. Factors are cached in /tmp/ilu_dag_M.npz.
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import fdlap  # noqa: E402


def factors(m):
    path = "/tmp/ilu_dag_%d.npz" % m
    if os.path.exists(path):
        z = np.load(path)
        L = sp.csr_matrix((z["Ld"], z["Li"], z["Lp"]), shape=(m * m, m * m))
        U = sp.csr_matrix((z["Ud"], z["Ui"], z["Up"]), shape=(m * m, m * m))
        return L, U, z["pr"], z["pc"]
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    t = time.time()
    ilu = spla.spilu(A.tocsc(), drop_tol=1e-3, fill_factor=15, diag_pivot_thresh=0.0)
    print("spilu %.1f s" % (time.time() - t))
    L, U = ilu.L.tocsr(), ilu.U.tocsr()
    np.savez(path, Ld=L.data, Li=L.indices, Lp=L.indptr, Ud=U.data, Ui=U.indices, Up=U.indptr,
             pr=ilu.perm_r, pc=ilu.perm_c)
    return L, U, ilu.perm_r, ilu.perm_c


def strict(T, lower):
    T = T.tocoo()
    keep = T.col < T.row if lower else T.col > T.row
    return sp.csr_matrix((T.data[keep], (T.row[keep], T.col[keep])), shape=T.shape)


_C = r"""
#include <stdint.h>
/* longest path (levels) and weighted longest path over a strictly triangular CSR factor */
void wlp(int64_t n, const int32_t *ip, const int32_t *ix, int lower, const int32_t *tile,
         double a, double b, double c, double *fin, int64_t *lev) {
    for (int64_t k = 0; k < n; ++k) {
        int64_t i = lower ? k : n - 1 - k;
        double t = 0.0; int64_t l = 0;
        for (int32_t e = ip[i]; e < ip[i + 1]; ++e) {
            int32_t j = ix[e];
            double u = fin[j] + (tile[i] == tile[j] ? a : b);
            if (u > t) t = u;
            if (lev[j] + 1 > l) l = lev[j] + 1;
        }
        fin[i] = t + c; lev[i] = l;
    }
}

/* list schedule: rows in solve-position order `ord`; row i belongs to workgroup wg[i] and is the
   pos[i]-th row of it; wave pos[i] % W of that workgroup runs its rows one after the other. */
double sim(int64_t n, const int32_t *ip, const int32_t *ix, const int64_t *ord, const int32_t *wg,
           const int64_t *pos, int W, double a, double b, double c, int64_t C, double *fin, double *wfree) {
    double mx = 0.0;
    for (int64_t k = 0; k < n; ++k) {
        int64_t i = ord[k];
        double t = wfree[(int64_t)wg[i] * W + pos[i] % W];
        for (int32_t e = ip[i]; e < ip[i + 1]; ++e) {
            int32_t j = ix[e];
            double u = fin[j] + ((wg[i] == wg[j] && pos[i] - pos[j] < C) ? a : b);
            if (u > t) t = u;
        }
        fin[i] = t + c;
        wfree[(int64_t)wg[i] * W + pos[i] % W] = t + c;
        if (t + c > mx) mx = t + c;
    }
    return mx;
}

/* the same with dynamic dealing: a workgroup's next row (in `ord`) goes to its earliest-free wave */
double simdyn(int64_t n, const int32_t *ip, const int32_t *ix, const int64_t *ord, const int32_t *wg,
              const int64_t *pos, int W, double a, double b, double c, int64_t C, double *fin, double *wfree) {
    double mx = 0.0;
    for (int64_t k = 0; k < n; ++k) {
        int64_t i = ord[k];
        double *wf = wfree + (int64_t)wg[i] * W;
        int best = 0;
        for (int w = 1; w < W; ++w) if (wf[w] < wf[best]) best = w;
        double t = wf[best];
        for (int32_t e = ip[i]; e < ip[i + 1]; ++e) {
            int32_t j = ix[e];
            double u = fin[j] + ((wg[i] == wg[j] && pos[i] - pos[j] < C) ? a : b);
            if (u > t) t = u;
        }
        fin[i] = t + c;
        wf[best] = t + c;
        if (t + c > mx) mx = t + c;
    }
    return mx;
}
"""


def simulate(S, lev, wg, W, a, b, c, C=1 << 40, dyn=False):
    """Time of the solve when workgroup wg[i]'s rows run in the order of the key `lev` (levels, or
    ASAP times) dealt round-robin (or dynamically) to W waves."""
    import ctypes
    n = S.shape[0]
    ord_ = np.lexsort((np.arange(n), lev)).astype(np.int64)     # key order (ties: index)
    wg = np.ascontiguousarray(wg, np.int32)
    # position of each row inside its workgroup, in level order
    srt = ord_[np.argsort(wg[ord_], kind="stable")]
    cnt = np.bincount(wg, minlength=int(wg.max()) + 1)
    starts = np.concatenate(([0], np.cumsum(cnt)[:-1]))
    pos = np.empty(n, np.int64)
    pos[srt] = np.arange(n) - np.repeat(starts, cnt)
    ip = np.ascontiguousarray(S.indptr, np.int32)
    ix = np.ascontiguousarray(S.indices, np.int32)
    fin = np.zeros(n)
    wfree = np.zeros((int(wg.max()) + 1) * W)
    P = ctypes.c_void_p
    f = _lib().simdyn if dyn else _lib().sim
    f.restype = ctypes.c_double
    return f(ctypes.c_int64(n), P(ip.ctypes.data), P(ix.ctypes.data), P(ord_.ctypes.data), P(wg.ctypes.data),
             P(pos.ctypes.data), ctypes.c_int(W), ctypes.c_double(a), ctypes.c_double(b), ctypes.c_double(c),
             ctypes.c_int64(C), P(fin.ctypes.data), P(wfree.ctypes.data))


def _lib():
    import ctypes
    import subprocess
    so = "/tmp/ilu_dag_c.so"
    if not os.path.exists(so):
        with open("/tmp/ilu_dag_c.c", "w") as f:
            f.write(_C)
        subprocess.check_call(["gcc", "-O2", "-std=c99", "-shared", "-fPIC", "/tmp/ilu_dag_c.c", "-o", so])
    return ctypes.CDLL(so)


def weighted_path(S, lower, tile, a, b, c):
    """(critical path with per-edge cost a (same tile) / b (other tile) + per-row cost c, levels)."""
    import ctypes
    n = S.shape[0]
    ip = np.ascontiguousarray(S.indptr, np.int32)
    ix = np.ascontiguousarray(S.indices, np.int32)
    tile = np.ascontiguousarray(tile, np.int32)
    fin = np.zeros(n)
    lev = np.zeros(n, np.int64)
    P = ctypes.c_void_p
    _lib().wlp(ctypes.c_int64(n), P(ip.ctypes.data), P(ix.ctypes.data), ctypes.c_int(int(lower)),
               P(tile.ctypes.data), ctypes.c_double(a), ctypes.c_double(b), ctypes.c_double(c),
               P(fin.ctypes.data), P(lev.ctypes.data))
    return float(fin.max()), lev


def _fin(S, lower, tile, a, b, c):
    import ctypes
    n = S.shape[0]
    ip = np.ascontiguousarray(S.indptr, np.int32)
    ix = np.ascontiguousarray(S.indices, np.int32)
    tile = np.ascontiguousarray(tile, np.int32)
    fin = np.zeros(n)
    lev = np.zeros(n, np.int64)
    P = ctypes.c_void_p
    _lib().wlp(ctypes.c_int64(n), P(ip.ctypes.data), P(ix.ctypes.data), ctypes.c_int(int(lower)),
               P(tile.ctypes.data), ctypes.c_double(a), ctypes.c_double(b), ctypes.c_double(c),
               P(fin.ctypes.data), P(lev.ctypes.data))
    return fin


def main():
    m = int(sys.argv[1])
    Ts = [int(t) for t in sys.argv[2:]] or [32, 64, 128]
    L, U, pr, pc = factors(m)
    n = m * m
    print("nnz L %d U %d" % (L.nnz, U.nnz), "perm_r==perm_c:", bool(np.array_equal(pr, pc)))
    Ls, Us = strict(L, True), strict(U, False)
    # grid point of every factor row: L row pr[i] <-> point i; U row pc[j] <-> point j
    ptL = np.empty(n, np.int64)
    ptL[pr] = np.arange(n)
    ptU = np.empty(n, np.int64)
    ptU[pc] = np.arange(n)
    for name, S, lower, pt in (("L", Ls, True, ptL), ("U", Us, False, ptU)):
        _, lev = weighted_path(S, lower, np.zeros(n, np.int32), 1.0, 1.0, 0.0)
        nl = int(lev.max()) + 1
        print("%s: levels %d, rows/level mean %.0f, entries/row %.1f" % (name, nl, n / nl, S.nnz / n))
        for a, b, c in ((0.1, 1.2, 0.15),):
            for P in (256, 512):
                wg = (pt * P) // n
                fin_t = _fin(S, lower, wg, a, b, c)
                print("  strips P=%d: level/rr %.2f level/dyn %.2f asap/rr %.2f asap/dyn %.2f | C=8192 asap/dyn %.2f" % (
                    P, simulate(S, lev, wg, 16, a, b, c) / 1e3, simulate(S, lev, wg, 16, a, b, c, dyn=True) / 1e3,
                    simulate(S, fin_t, wg, 16, a, b, c) / 1e3, simulate(S, fin_t, wg, 16, a, b, c, dyn=True) / 1e3,
                    simulate(S, fin_t, wg, 16, a, b, c, 8192, dyn=True) / 1e3))
            line = "  strips of the original index, a=%.2f b=%.2f c=%.2f:" % (a, b, c)
            for P in (256, 512, 1024):
                line += " P=%d %.2f" % (P, simulate(S, lev, (pt * P) // n, 16, a, b, c) / 1e3)
                if P == 256:
                    for C in (4096, 8192, 12288):
                        line += " (C=%d %.2f)" % (C, simulate(S, lev, (pt * P) // n, 16, a, b, c, C) / 1e3)
                if P == 512:
                    line += " (8 waves %.2f)" % (simulate(S, lev, (pt * P) // n, 8, a, b, c) / 1e3)
            print(line + " | sync-free at 1.19 us/level %.2f ms" % (nl * 1.19e-3))
        for T in Ts if len(sys.argv) > 2 else []:
            ty, tx = (pt // m) // T, (pt % m) // T
            tile = ty * ((m + T - 1) // T) + tx
            cross = 0
            rows = np.repeat(np.arange(n), np.diff(S.indptr))
            cross = int(np.count_nonzero(tile[rows] != tile[S.indices]))
            for a, b, c in ((0.1, 1.2, 0.15), (0.2, 1.5, 0.2)):
                cp, _ = weighted_path(S, lower, tile, a, b, c)
                nt = int(tile.max()) + 1
                line = "  T=%4d tiles %6d cross %.3f a=%.2f b=%.2f c=%.2f: path %.2f ms" % (
                    T, nt, cross / max(1, S.nnz), a, b, c, cp / 1e3)
                for P in (256, 512):
                    if nt >= P:
                        # tiles -> workgroups: tile t -> t % P (spread) and blocks of consecutive tiles
                        line += " | P=%d spread %.2f" % (P, simulate(S, lev, tile % P, 16, a, b, c) / 1e3)
                        line += " block %.2f" % (simulate(S, lev, (tile * P) // nt, 16, a, b, c) / 1e3)
                print(line)


if __name__ == "__main__":
    main()
