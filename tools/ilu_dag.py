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

/* chains: rows in solve order; row i extends the chain of its latest-finishing dependency p when p
   is still that chain's tail (then it runs right after p on p's wave: in-chain hop a, x_p from a
   register), else (mode 1) the latest-finishing dependency that is a tail, else it starts a chain;
   every other dependency costs b (a published value). c = per-row cost. Waves unbounded; returns the
   makespan, writes the number of chains and the longest one. */
double chains(int64_t n, const int32_t *ip, const int32_t *ix, int lower, int mode, double a, double b, double c,
              double *fin, int8_t *tail, int32_t *clen, int64_t *stats) {
    double mx = 0.0; int64_t nch = 0, longest = 0;
    for (int64_t k = 0; k < n; ++k) {
        int64_t i = lower ? k : n - 1 - k;
        int64_t best = -1, bt = -1; double tb = -1.0, tt = -1.0;
        for (int32_t e = ip[i]; e < ip[i + 1]; ++e) {
            int32_t j = ix[e];
            if (fin[j] > tb) { tb = fin[j]; best = j; }
            if (tail[j] && fin[j] > tt) { tt = fin[j]; bt = j; }
        }
        int64_t p = (best >= 0 && tail[best]) ? best : (mode == 1 ? bt : -1);
        double t = 0.0;
        for (int32_t e = ip[i]; e < ip[i + 1]; ++e) {
            int32_t j = ix[e];
            double u = fin[j] + (j == p ? a : b);
            if (u > t) t = u;
        }
        if (p >= 0) { tail[p] = 0; clen[i] = clen[p] + 1; } else { clen[i] = 1; ++nch; }
        if (clen[i] > longest) longest = clen[i];
        tail[i] = 1;
        fin[i] = t + c;
        if (fin[i] > mx) mx = fin[i];
    }
    stats[0] = nch; stats[1] = longest;
    return mx;
}

/* Wave-chained sync-free order: positions k = 0, 1, ... are filled greedily in a topological order
   and dealt round-robin (wave k mod W, as sptrsv_kernel deals them). Position k preferably takes the
   designated child of the row at position k - W (the previous row of the same wave) when all its
   parents are placed, so that dependency is a register hand-off; otherwise the ready row of lowest
   level (index order on ties). Deadlock-free by construction: every row follows all its parents.
   Then the timing: per row c, a dependency on the same wave's previous row a, any other b. */
#include <stdlib.h>
typedef struct { int64_t key; int64_t row; } hitem;
static void hpush(hitem *h, int64_t *sz, hitem v) {
    int64_t i = (*sz)++;
    while (i > 0) { int64_t p = (i - 1) / 2; if (h[p].key <= v.key) break; h[i] = h[p]; i = p; }
    h[i] = v;
}
static hitem hpop(hitem *h, int64_t *sz) {
    hitem top = h[0], v = h[--(*sz)];
    int64_t i = 0;
    for (;;) { int64_t l = 2 * i + 1, r = l + 1, m = i;
        hitem mv = v;
        if (l < *sz && h[l].key < mv.key) { m = l; mv = h[l]; }
        if (r < *sz && h[r].key < mv.key) { m = r; mv = h[r]; }
        if (m == i) break; h[i] = h[m]; i = m; }
    h[i] = v;
    return top;
}
/* cp/ci: children CSR (parents -> children); lev: levels; desig[p] = designated child or -1 */
double wave_chain(int64_t n, const int32_t *ip, const int32_t *ix, const int32_t *cp, const int32_t *ci,
                  const int64_t *lev, const int32_t *desig, int64_t W, double a, double b, double c,
                  int64_t *order, double *fin, int64_t *stats) {
    int32_t *npar = (int32_t *)malloc(sizeof(int32_t) * n);
    int8_t *placed = (int8_t *)calloc(n, 1);
    int64_t *pos = (int64_t *)malloc(sizeof(int64_t) * n);
    hitem *h = (hitem *)malloc(sizeof(hitem) * (n + 1));
    double *wfree = (double *)calloc(W, sizeof(double));
    int64_t sz = 0, chained = 0;
    for (int64_t i = 0; i < n; ++i) {
        npar[i] = ip[i + 1] - ip[i];
        if (npar[i] == 0) { hitem v = {lev[i] * n + i, i}; hpush(h, &sz, v); }
    }
    double mx = 0.0;
    for (int64_t k = 0; k < n; ++k) {
        int64_t r = -1;
        if (k >= W) { int64_t prev = order[k - W]; int64_t d = desig[prev]; if (d >= 0 && npar[d] == 0 && !placed[d]) r = d; }
        if (r < 0) { do { r = hpop(h, &sz).row; } while (placed[r]); } else ++chained;
        placed[r] = 1; order[k] = r; pos[r] = k;
        for (int32_t e = cp[r]; e < cp[r + 1]; ++e) { int32_t ch = ci[e];
            if (--npar[ch] == 0) { hitem v = {lev[ch] * n + ch, ch}; hpush(h, &sz, v); } }
        /* timing */
        int64_t w = k % W; double t = wfree[w];
        for (int32_t e = ip[r]; e < ip[r + 1]; ++e) { int32_t j = ix[e];
            double u = fin[j] + (pos[j] == k - W ? a : b); if (u > t) t = u; }
        fin[r] = t + c; wfree[w] = t + c; if (fin[r] > mx) mx = fin[r];
    }
    stats[0] = chained;
    free(npar); free(placed); free(pos); free(h); free(wfree);
    return mx;
}

/* chain ids and [start, end] of every chain of the schedule above (call after `chains`) */
void chain_ids(int64_t n, const int32_t *ip, const int32_t *ix, int lower, int mode, const double *fin,
               int32_t *cid, double *cstart, double *cend, int8_t *tail) {
    int32_t nch = 0;
    for (int64_t k = 0; k < n; ++k) {
        int64_t i = lower ? k : n - 1 - k;
        int64_t best = -1, bt = -1; double tb = -1.0, tt = -1.0;
        for (int32_t e = ip[i]; e < ip[i + 1]; ++e) {
            int32_t j = ix[e];
            if (fin[j] > tb) { tb = fin[j]; best = j; }
            if (tail[j] && fin[j] > tt) { tt = fin[j]; bt = j; }
        }
        int64_t p = (best >= 0 && tail[best]) ? best : (mode == 1 ? bt : -1);
        if (p >= 0) { tail[p] = 0; cid[i] = cid[p]; }
        else { cid[i] = nch; cstart[nch] = fin[i]; ++nch; }
        cend[cid[i]] = fin[i];
        tail[i] = 1;
    }
}
"""


def chain_sim(S, lower, mode, a, b, c):
    """(makespan us, chains, longest chain) of the chain schedule (see `chains` above)."""
    import ctypes
    n = S.shape[0]
    ip = np.ascontiguousarray(S.indptr, np.int32)
    ix = np.ascontiguousarray(S.indices, np.int32)
    fin = np.zeros(n)
    tail = np.zeros(n, np.int8)
    clen = np.zeros(n, np.int32)
    st = np.zeros(2, np.int64)
    P = ctypes.c_void_p
    f = _lib().chains
    f.restype = ctypes.c_double
    t = f(ctypes.c_int64(n), P(ip.ctypes.data), P(ix.ctypes.data), ctypes.c_int(int(lower)), ctypes.c_int(mode),
          ctypes.c_double(a), ctypes.c_double(b), ctypes.c_double(c), P(fin.ctypes.data), P(tail.ctypes.data),
          P(clen.ctypes.data), P(st.ctypes.data))
    return t, int(st[0]), int(st[1])


def wave_chain_sim(S, lower, W, a, b, c, desig_mode="level"):
    """Makespan (us) of the wave-chained sync-free order (see `wave_chain`), and the share of rows
    that follow their designated parent on the same wave."""
    import ctypes
    n = S.shape[0]
    # solve-order indexing: row i of the lower solve is node i; the upper solve runs n-1..0
    T = S if lower else S[::-1, ::-1].tocsr()
    T.sort_indices()
    ip = np.ascontiguousarray(T.indptr, np.int32)
    ix = np.ascontiguousarray(T.indices, np.int32)
    _, lev = weighted_path(T, True, np.zeros(n, np.int32), 1.0, 1.0, 0.0)
    C = T.T.tocsr()
    cp = np.ascontiguousarray(C.indptr, np.int32)
    ci = np.ascontiguousarray(C.indices, np.int32)
    # designated child of p: the first child (index order) whose level is lev[p] + 1 and for which p
    # is its highest-index parent at level lev[child] - 1 (one child per parent)
    rows = np.repeat(np.arange(n), np.diff(ip))
    par = ix
    crit = lev[par] == lev[rows] - 1
    best = np.full(n, -1, np.int64)
    np.maximum.at(best, rows[crit], par[crit])       # each row's critical parent (highest index)
    desig = np.full(n, -1, np.int32)
    kids = np.nonzero(best >= 0)[0]
    # first child per parent
    ordk = kids[np.argsort(best[kids], kind="stable")]
    bp = best[ordk]
    first = np.ones(len(ordk), bool)
    first[1:] = bp[1:] != bp[:-1]
    desig[bp[first]] = ordk[first]
    order = np.zeros(n, np.int64)
    fin = np.zeros(n)
    st = np.zeros(2, np.int64)
    P = ctypes.c_void_p
    f = _lib().wave_chain
    f.restype = ctypes.c_double
    t = f(ctypes.c_int64(n), P(ip.ctypes.data), P(ix.ctypes.data), P(cp.ctypes.data), P(ci.ctypes.data),
          P(lev.ctypes.data), P(desig.ctypes.data), ctypes.c_int64(W), ctypes.c_double(a), ctypes.c_double(b),
          ctypes.c_double(c), P(order.ctypes.data), P(fin.ctypes.data), P(st.ctypes.data))
    return t, st[0] / n


def chain_concurrency(S, lower, mode, a, b, c):
    """Most chains alive at once in the unbounded chain schedule (each holds a wave)."""
    import ctypes
    n = S.shape[0]
    ip = np.ascontiguousarray(S.indptr, np.int32)
    ix = np.ascontiguousarray(S.indices, np.int32)
    fin = np.zeros(n)
    tail = np.zeros(n, np.int8)
    clen = np.zeros(n, np.int32)
    st = np.zeros(2, np.int64)
    P = ctypes.c_void_p
    lib = _lib()
    lib.chains.restype = ctypes.c_double
    lib.chains(ctypes.c_int64(n), P(ip.ctypes.data), P(ix.ctypes.data), ctypes.c_int(int(lower)), ctypes.c_int(mode),
               ctypes.c_double(a), ctypes.c_double(b), ctypes.c_double(c), P(fin.ctypes.data), P(tail.ctypes.data),
               P(clen.ctypes.data), P(st.ctypes.data))
    nch = int(st[0])
    cid = np.zeros(n, np.int32)
    cs, ce = np.zeros(nch), np.zeros(nch)
    tail[:] = 0
    lib.chain_ids(ctypes.c_int64(n), P(ip.ctypes.data), P(ix.ctypes.data), ctypes.c_int(int(lower)), ctypes.c_int(mode),
                  P(fin.ctypes.data), P(cid.ctypes.data), P(cs.ctypes.data), P(ce.ctypes.data), P(tail.ctypes.data))
    ev = np.concatenate([np.stack([cs - c, np.ones(nch)], 1), np.stack([ce, -np.ones(nch)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    return int(np.cumsum(ev[:, 1]).max()), np.bincount(np.bincount(cid))


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
    so = "/tmp/ilu_dag_c2.so"
    if not os.path.exists(so):
        with open("/tmp/ilu_dag_c2.c", "w") as f:
            f.write(_C)
        subprocess.check_call(["gcc", "-O2", "-std=c99", "-shared", "-fPIC", "/tmp/ilu_dag_c2.c", "-o", so])
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
        if os.environ.get("WAVECHAIN"):
            for W in (1024, 2048, 4096, 7168):
                for a, b, c in ((0.0, 1.0, 0.2), (0.0, 1.0, 0.35)):
                    t, share = wave_chain_sim(S, lower, W, a, b, c)
                    t0, _ = wave_chain_sim(S, lower, W, b, b, c)   # no register hand-off: plain sync-free
                    print("  wave-chain W=%d a=%.2f b=%.2f c=%.2f: %.2f ms (chained rows %.2f) vs sync-free %.2f ms"
                          % (W, a, b, c, t / 1e3, share, t0 / 1e3))
            continue
        if os.environ.get("CHAINS"):
            for mode in (0, 1):
                for a, b, c in ((0.0, 1.1, 0.15), (0.0, 1.1, 0.3), (0.0, 0.9, 0.2)):
                    t, nch, lg = chain_sim(S, lower, mode, a, b, c)
                    print("  chains mode %d a=%.2f b=%.2f c=%.2f: %.2f ms, %d chains, longest %d (sync-free at b+c/level %.2f ms)"
                          % (mode, a, b, c, t / 1e3, nch, lg, nl * (b + c) / 1e3))
                    if a == 0.0 and c == 0.15:
                        conc, hist = chain_concurrency(S, lower, mode, a, b, c)
                        print("    max chains alive at once %d; chains of length 1/2/3/4+: %s" % (
                            conc, [int(hist[1]) if len(hist) > 1 else 0, int(hist[2]) if len(hist) > 2 else 0,
                                   int(hist[3]) if len(hist) > 3 else 0, int(hist[4:].sum())]))
            continue
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
