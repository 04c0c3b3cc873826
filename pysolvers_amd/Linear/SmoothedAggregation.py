"""Smoothed-aggregation coarsening (SmoothedAggregation.py:13-229), O(nnz) host setup.

The reference's BuildAggregates is quadratic (phase 2 scans every aggregate for every remaining
node; 253 s at FD 512^2). Here aggregation and the filtered matrix come from
``psk_sa_aggregate`` (C++, pysolvers_amd/csrc/amg.hip) with identical results, and the remaining
steps use the same scipy operations the reference uses, so P, R and every coarse operator are
bit-identical to the reference's (tests: oracle/amg.py is pinned against the reference; the CPU
tests check this module against oracle/amg.py).
"""
import ctypes

import numpy as np
import scipy.sparse as sp

from .. import _native as N
from .MLHierarchy import MLHierarchy


def default_tol(lvl):
    return 0.08 * (0.5) ** (lvl - 1)          # Vanek's default (:62-63)


class SmoothedAggregationMLHierarchy(MLHierarchy):
    """SmoothedAggregation.py:13-31. ``tol`` is stored and, as in the reference, not used: every
    level is coarsened with the default tolerance of its level number (SA_coarsen passes only
    lvl to BuildAggregates, :218)."""

    def __init__(self, A_fine, numLevels=2, tol=None, normalize=True):
        super().__init__(numLevels=numLevels, normalize=normalize)
        self.tol = tol
        self.normalize = normalize
        self._setFineMatrix(sp.csr_matrix(A_fine))
        self._aggregates = [None] * numLevels
        for lev in reversed(range(numLevels - 1)):
            I_up = self.makeProlongator(lev)
            self._setUpdate(lev, I_up)

    def makeProlongator(self, lev):
        I_up, agg = SA_coarsen(self.matrix(lev + 1), tol=self.tol, lvl=lev + 1)
        self._aggregates[lev] = agg
        return I_up


def BuildAggregates(A, lvl=1):
    """(agg, count, Af_values): aggregate index per node in the reference's list order, and the
    filtered matrix values (BuildAggregates :57-143 + BuildFilteredMatrix :157-183)."""
    A = sp.csr_matrix(A)
    n = A.shape[0]
    indptr = np.ascontiguousarray(A.indptr, dtype=np.int32)
    indices = np.ascontiguousarray(A.indices, dtype=np.int32)
    data = np.ascontiguousarray(A.data, dtype=np.float64)
    agg = np.empty(n, dtype=np.int32)
    afv = np.empty(data.shape[0], dtype=np.float64)
    count = ctypes.c_int64()
    N.check(N.lib.psk_sa_aggregate(n, N.ptr(indptr), N.ptr(indices), N.ptr(data), default_tol(lvl), N.ptr(agg),
                                   ctypes.byref(count), N.ptr(afv)), "psk_sa_aggregate")
    return agg, int(count.value), afv


def SmoothProlongator(Phat, A, Af, omega=(2 / 3)):
    """P = (I - omega D^-1 A_f) P_hat, elementwise in the reference's order (:185-205)."""
    S = omega * Af
    dA = A.diagonal()
    rows = np.repeat(np.arange(S.shape[0]), np.diff(S.indptr))
    v = S.data / dA[rows]
    S.data[:] = np.where(S.indices == rows, 1 - v, -v)
    return S.dot(Phat)


def SA_coarsen(A, tol=None, lvl=1):
    """(P, agg) for one level (:208-229); agg[i] = aggregate (coarse node) of fine node i."""
    A = sp.csr_matrix(A)
    n = A.shape[0]
    agg, count, afv = BuildAggregates(A, lvl=lvl)
    Phat = sp.csr_matrix((np.ones(n), agg, np.arange(n + 1, dtype=np.int32)), shape=(n, count))   # :145-155
    Af = sp.csr_matrix((afv, A.indices.copy(), A.indptr.copy()), shape=A.shape)
    P = SmoothProlongator(Phat, A, Af)
    return P.tocsr(), agg
