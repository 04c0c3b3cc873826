"""AMG preconditioner (AMGPreconditioner.py:1-51): smoothed-aggregation V-cycles on the GPU.

``AMG(numIters, numLevels, nuPre, nuPost, smoother).form(A)`` builds the hierarchy on the host
(SmoothedAggregation.py, O(nnz), bit-identical P / R / A_k to the reference), uploads every level
once, and ``apply(v)`` = AMGVCycleSolver.solve(A, v) with CommonSolverArgs(maxiter=numIters,
failOnMaxiter=False) (VCycleSolver.py:52-95) runs entirely on the device (psk_prec_create_amg,
pysolvers_amd/csrc/amg.hip): numIters V-cycles from x0 = v, early exit on ||v - A x|| < 1e-8 ||v||.

Level operators: SpMV (bit-identical stored-order sums) for A_k, R_k, P_k; smoothing sweeps
x <- x + S^-1 (f - A x) with S^-1 = DInv* (Jacobi) or triu(A_k)^-1 (Gauss-Seidel, sync-free
triangular solve); the coarsest level is spsolve(A_0, f) (VCycleManager.py:34-37; the reference
refactors A_0 on every call, same factors each time). Since round 5 that solve is a streamed GEMV over
A_0^-1, formed once on the device (coarse="dense", pysolvers_amd/csrc/dense.hip): one HBM-bound pass
instead of a sparse triangular-solve chain thousands of dependency levels deep (4.84 -> ~0.4 ms at
-FD 8192^2, A_0 16,642^2); it agrees with SuperLU's solve to ~1e-15 relative (tests pin 1e-12).
coarse="lu" keeps SuperLU's factors of A_0 computed once on the host as two device triangular solves.
"auto" (default) takes the dense inverse up to 32,768 unknowns and falls back to the factors when the
inverse cannot be formed (A_0 singular, rocSOLVER absent).
"""
import ctypes

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from .. import _native as N
from .ClassicSmoothers import GaussSeidelSmoother, JacobiSmoother
from .DeviceMatrix import DeviceCSR
from .Preconditioner import DeviceOperator, GenericPreconditioner
from .PreconditionerType import PreconditionerType
from .SmoothedAggregation import SmoothedAggregationMLHierarchy
from .TriangularSolve import superlu_transposed_solver


class AMG(PreconditionerType):
    def __init__(self, numIters=5, numLevels=2, nuPre=2, nuPost=2, smoother=GaussSeidelSmoother, coarse="auto",
                 coarse_refine=0):
        self.numIters = numIters
        self.numLevels = numLevels
        self.nuPre = nuPre
        self.nuPost = nuPost
        self.smoother = smoother
        self.coarse = coarse
        self.coarse_refine = coarse_refine

    def form(self, A):
        return AMGPreconditioner(A, numIters=self.numIters, numLevels=self.numLevels, nuPre=self.nuPre,
                                 nuPost=self.nuPost, smoother=self.smoother, coarse=self.coarse,
                                 coarse_refine=self.coarse_refine)


def coarse_factor(A_c):
    """The factorisation spsolve(A_c, f) (VCycleManager.py:36) performs, once: spsolve sorts A_c
    (sum_duplicates), hands the CSR arrays to SuperLU as the CSC of A_c^T and solves transposed;
    splu of that same matrix with COLAMD gives the same factors (checked bitwise in the tests)."""
    Ac = sp.csr_matrix(A_c, copy=True)
    Ac.sum_duplicates()
    n = Ac.shape[0]
    AA = sp.csc_matrix((Ac.data, Ac.indices, Ac.indptr), shape=(n, n))
    return spla.splu(AA, permc_spec='COLAMD')


def coarse_solver(A_c):
    """(device operator x = A_c^-1 f, SuperLU object)."""
    lu = coarse_factor(A_c)
    return superlu_transposed_solver(lu), lu


DENSE_COARSE_MAX = 32768   # kDenseMaxN (psk_internal.hpp): 8.6 GB of inverse


class DenseInverseSolver(DeviceOperator):
    """x = A^-1 f through A's explicit inverse on the device (psk_prec_create_dense_inverse): formed once
    (rocSOLVER getrf/getri), each apply one streamed GEMV plus `refine` steps x += A^-1 (f - A x)."""

    device_kind = N.PSK_PREC_DENSE

    def __init__(self, A, refine=0):
        self._A = A if isinstance(A, DeviceCSR) else DeviceCSR.from_scipy(sp.csr_matrix(A))   # borrowed
        self.n = self._A.n
        self.refine = int(refine)
        h = ctypes.c_void_p()
        N.check(N.lib.psk_prec_create_dense_inverse(self._A.handle, self.refine, ctypes.byref(h)),
                "psk_prec_create_dense_inverse")
        self._h = h

    def apply(self, vec):
        return self._device_apply(vec)


class AMGPreconditioner(DeviceOperator, GenericPreconditioner):
    device_kind = N.PSK_PREC_AMG

    def __init__(self, A, numIters=5, numLevels=2, nuPre=2, nuPost=2, smoother=GaussSeidelSmoother, tau=1.0e-8,
                 coarse="auto", coarse_refine=None):
        if smoother not in (GaussSeidelSmoother, JacobiSmoother):
            raise TypeError("AMG smoother must be GaussSeidelSmoother or JacobiSmoother")
        if coarse not in ("auto", "dense", "lu"):
            raise ValueError("AMG coarse must be 'auto', 'dense' or 'lu'")
        dA = A if isinstance(A, DeviceCSR) else DeviceCSR.from_scipy(A)
        Ah = A.to_scipy() if isinstance(A, DeviceCSR) else sp.csr_matrix(A)
        self.n = Ah.shape[0]
        self.numIters, self.numLevels, self.nuPre, self.nuPost = numIters, numLevels, nuPre, nuPost
        self.mlh = SmoothedAggregationMLHierarchy(Ah, numLevels=numLevels)
        L = numLevels
        # device copies; the finest level is the caller's matrix
        self._A = [DeviceCSR.from_scipy(self.mlh.matrix(k)) for k in range(L - 1)] + [dA]
        self._P = [DeviceCSR.from_scipy(self.mlh.update(k), rectangular=True) for k in range(L - 1)]
        self._R = [DeviceCSR.from_scipy(self.mlh.downdate(k), rectangular=True) for k in range(L - 1)]
        self._S = [None] + [smoother(self.mlh.matrix(k), device_A=self._A[k]) for k in range(1, L)]
        self._coarse, self._lu, self.coarse_kind = None, None, "lu"
        # auto: the dense inverse with one refinement step x += A_0^-1 (f - A_0 x) (the inverse's forward
        # error grows with cond(A_0) where spsolve's LU is backward stable; one step brings it back to the LU's
        # level at 0.78 instead of 0.40 ms per solve, against 4.84 for the factors), and only when the inverse
        # takes at most half of the free device memory (psk_prec_create_dense_inverse refuses it otherwise)
        if coarse_refine is None:
            coarse_refine = 1 if coarse == "auto" else 0
        if coarse == "dense" or (coarse == "auto" and 0 < self._A[0].n <= DENSE_COARSE_MAX):
            try:
                self._coarse = DenseInverseSolver(self._A[0], refine=coarse_refine)
                self.coarse_kind = "dense"
            except N.PskError as e:   # singular A_0, rocSOLVER absent, out of memory: the factors instead
                if coarse == "dense" or e.code in (N.PSK_ERR_HIP, N.PSK_ERR_RCCL):
                    raise
        if self._coarse is None:
            self._coarse, self._lu = coarse_solver(self.mlh.matrix(0))
        pa, ka = N.handle_array([d.handle for d in self._A])
        pp, kp = N.handle_array([d.handle for d in self._P])
        pr, kr = N.handle_array([d.handle for d in self._R])
        ps, ks = N.handle_array([None] + [s.operator.device_handle for s in self._S[1:]])
        h = ctypes.c_void_p()
        N.check(N.lib.psk_prec_create_amg(L, pa, pp, pr, ps, self._coarse.device_handle, int(numIters), int(nuPre),
                                          int(nuPost), float(tau), ctypes.byref(h)), "psk_prec_create_amg")
        self._h = h

    def apply(self, vec):
        return self._device_apply(vec)

    def levels(self):
        """Sizes n_0 (coarsest) .. n_{L-1} (finest)."""
        return [d.n for d in self._A]
