"""Device triangular-solve chains (psk_prec_create_trisolve) built from host scipy factors.

One operator covers every triangular apply the reference's preconditioners perform through SuperLU
or spsolve_triangular: ILU.solve (ILUTPreconditioner.py:70-78), the IC pair L^-1 then L^-T
(ICPreconditioner.py:58-63), the Gauss-Seidel smoother's triu(A)^-1 (ClassicSmoothers.py:28-36) and
the AMG coarse solve spsolve(A_c, f) (VCycleManager.py:34-37):

    out = (U^-1 L^-1 v[gather_in])[gather_out]

with either factor optional and each factor unit- or non-unit-diagonal.
"""
import ctypes

import numpy as np
import scipy.sparse as sp

from .. import _native as N
from .Preconditioner import DeviceOperator, GenericPreconditioner


def _csr_arrays(M):
    M = sp.csr_matrix(M)
    return (np.ascontiguousarray(M.indptr, dtype=np.int32), np.ascontiguousarray(M.indices, dtype=np.int32),
            np.ascontiguousarray(M.data, dtype=np.float64))


def inverse_permutation(p):
    p = np.asarray(p, dtype=np.int64)
    inv = np.empty_like(p)
    inv[p] = np.arange(p.shape[0])
    return inv


class TriangularSolveChain(DeviceOperator, GenericPreconditioner):
    """out = (U^-1 L^-1 v[gather_in])[gather_out] on the device.

    L: lower-triangular CSR (or None), U: upper-triangular CSR (or None); *_unit: unit diagonal
    (stored diagonal entries ignored), else the stored diagonal divides. Rows of each factor are
    solved by one wave each, in a host-computed dependency-level order (see pysolvers_amd/csrc/ilu.hip).
    """

    device_kind = N.PSK_PREC_ILU

    def __init__(self, n, L=None, l_unit=False, U=None, u_unit=False, gather_in=None, gather_out=None):
        self.n = int(n)
        keep = []

        def arrs(M):
            if M is None:
                return [None, None, None]
            a = _csr_arrays(M)
            keep.extend(a)
            return [N.ptr(x) for x in a]

        def perm(p):
            if p is None:
                return None
            a = np.ascontiguousarray(p, dtype=np.int32)
            keep.append(a)
            return N.ptr(a)

        h = ctypes.c_void_p()
        N.check(N.lib.psk_prec_create_trisolve(self.n, *arrs(L), int(bool(l_unit)), *arrs(U), int(bool(u_unit)),
                                               perm(gather_in), perm(gather_out), ctypes.byref(h)),
                "psk_prec_create_trisolve")
        self._h = h

    def apply(self, vec):
        return self._device_apply(vec)

    def schedule(self, which, set=None):
        """dict(schedule, blocks, ring_words, est_syncfree_us, est_band_us) of factor `which` ('L' or
        'U'); set='syncfree' / 'band' / 'lds' / 'grid' / 'part' / 'levels' forces a schedule
        (psk_prec_trisolve_schedule)."""
        code = {None: -1, "syncfree": 0, "band": 1, "lds": 2, "grid": 3, "part": 4, "levels": 5}[set]
        sc, bl, rw, e0, e1 = N.I32(), N.I64(), N.I32(), N.F64(), N.F64()
        N.check(N.lib.psk_prec_trisolve_schedule(self._h, {"L": 0, "U": 1}[which], code, ctypes.byref(sc),
                                                 ctypes.byref(bl), ctypes.byref(rw), ctypes.byref(e0),
                                                 ctypes.byref(e1)), "psk_prec_trisolve_schedule")
        return dict(schedule=("syncfree", "band", "lds", "grid", "part", "levels")[sc.value], blocks=bl.value,
                    ring_words=rw.value,
                    est_syncfree_us=e0.value, est_band_us=e1.value)

    def grid_info(self, which):
        """Grid-schedule shape of factor `which` (psk_prec_trisolve_grid_info): dict(w, H, sigma2, phase, off,
        steps, dict_records) — position y*w + x - off runs at step x + ((sigma2*y + phase) >> 1)."""
        out = (N.I64 * 7)()
        N.check(N.lib.psk_prec_trisolve_grid_info(self._h, {"L": 0, "U": 1}[which], out), "psk_prec_trisolve_grid_info")
        return dict(zip(("w", "H", "sigma2", "phase", "off", "steps", "dict_records"), list(out)))


def grid_plan(T, upper):
    """The grid plan (psk_trisolve_grid_plan, host only) of triangular factor T (CSR with its diagonal;
    upper: solved from the last row up): dict(w, H, sigma2, phase, off, steps, K), or None when T is not
    a 2-D stencil. Position y*w + x - off runs at step x + ((sigma2*y + phase) >> 1)."""
    T = sp.csr_matrix(T)
    rp = np.ascontiguousarray(T.indptr, dtype=np.int32)
    ci = np.ascontiguousarray(T.indices, dtype=np.int32)
    va = np.ascontiguousarray(T.data, dtype=np.float64)
    out = (N.I64 * 7)()
    rc = N.lib.psk_trisolve_grid_plan(T.shape[0], N.ptr(rp), N.ptr(ci), N.ptr(va), 1 if upper else 0, out)
    if rc == -5:   # PSK_ERR_UNSUPPORTED
        return None
    N.check(rc, "psk_trisolve_grid_plan")
    return dict(zip(("w", "H", "sigma2", "phase", "off", "steps", "K"), list(out)))


def superlu_transposed_solver(lu):
    """x = lu.solve(b, trans='T') as a chain: with Pr B Pc = L U, B^T x = b gives
    x = Pr^T L^-T U^-T Pc^T b, i.e. gather_in = perm_c^-1, lower = U^T (non-unit),
    upper = L^T (unit), gather_out = perm_r. A CSC factor's arrays read as CSR are its transpose."""
    n = lu.shape[0]
    Ut = sp.csr_matrix((lu.U.data, lu.U.indices, lu.U.indptr), shape=(n, n))
    Lt = sp.csr_matrix((lu.L.data, lu.L.indices, lu.L.indptr), shape=(n, n))
    return TriangularSolveChain(n, L=Ut, l_unit=False, U=Lt, u_unit=True,
                                gather_in=inverse_permutation(lu.perm_c), gather_out=lu.perm_r)
