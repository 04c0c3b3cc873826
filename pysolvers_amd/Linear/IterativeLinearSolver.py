"""Iterative-solver factory/base classes and ``mvmult`` (IterativeLinearSolver.py:1-106).

``IterativeLinearSolver._device_solve`` is the one place where the Python
layer crosses into libpsk: it puts A in HBM (``DeviceCSR``), forms the
preconditioner through the plugin API (``PreconditionerType.form``), hands
the whole Krylov loop to ``psk_pcg`` / ``psk_gmres`` and turns the returned
psk_result into the SolveStatus the reference would have returned.
"""
import ctypes

import numpy as np
import scipy.sparse as sp

from .. import _native as N
from ..IterativeSolver import CommonSolverArgs, IterativeSolver, SolveStatus
from .DeviceMatrix import DeviceCSR, DeviceVector, as_device_matrix, is_device_vector, spmv, torch_stream_ready
from .LinearSolver import LinearSolver, LinearSolverType
from .PreconditionerType import IdentityPreconditionerType


class IterativeLinearSolverType(LinearSolverType):
    """Factory base (IterativeLinearSolver.py:32-54)."""

    def __init__(self, control=CommonSolverArgs(), precond=IdentityPreconditionerType(), name=''):
        super().__init__(name)
        self._control = control
        self._precondType = precond

    def precond(self):
        return self._precondType

    def control(self):
        return self._control


class IterativeLinearSolver(LinearSolver, IterativeSolver):
    """Solver base (IterativeLinearSolver.py:60-86) + the device driver."""

    _entry = None          # "psk_pcg" / "psk_gmres"

    def __init__(self, control, precond=IdentityPreconditionerType(), name=''):
        LinearSolver.__init__(self, name=name)
        IterativeSolver.__init__(self, control=control, name=name)
        self._precondType = precond
        self._precFrozen = False
        self.precond = None
        self._dA = None
        self._dA_src = None
        self.time_kernels = False      # HIP-event timing of the SpMV launches (bench)

    def precondType(self):
        return self._precondType

    def setTolerance(self, tau):
        super().setTolerance(tau)

    def freezePrec(self):
        self._precFrozen = True

    def unfreezePrec(self):
        self._precFrozen = False

    def precFrozen(self):
        return self._precFrozen

    def _restart(self):
        return 0

    # -----------------------------------------------------------------------------------------
    def _device_matrix(self, A):
        if isinstance(A, DeviceCSR):
            return A
        if self.matrixFrozen() and self._dA is not None and self._dA_src is A:
            return self._dA
        dA = DeviceCSR.from_scipy(A)
        self._dA, self._dA_src = dA, A
        return dA

    def _device_solve(self, A, b):
        n, nc = A.shape
        if not (isinstance(A, DeviceCSR) and A.comm is not None):
            assert n == nc                                   # PCGSolver.py:79-81
        assert n == len(b)                                   # PCGSolver.py:83
        self._check_norm()
        dA = self._device_matrix(A)
        if self.precond is None or not self.precFrozen():   # PCGSolver.py:92-94
            self.precond = self.precondType().form(dA)
        kind = getattr(self.precond, "device_kind", None)
        if kind is None:
            raise TypeError("%s: preconditioner %r has no device implementation; available: "
                            "IdentityPreconditionerType, JacobiPreconditionerType, RightILUT, RightIC, AMG"
                            % (self.name(), type(self.precond).__name__))
        ph = None if kind == N.PSK_PREC_IDENTITY else self.precond.device_handle

        maxiter = int(self.maxiter())
        ctl = N.PskCtl(maxiter=maxiter, tau=float(self.tau()), fail_on_maxiter=int(bool(self.failOnMaxiter())),
                       restart=int(self._restart()), check_every=0, time_kernels=int(bool(self.time_kernels)))
        res = N.PskResult()
        hist = np.zeros(max(maxiter, 1), dtype=np.float64)
        if isinstance(b, DeviceVector):
            x, loc, bp = DeviceVector(n), N.PSK_DEVICE, b
        elif is_device_vector(b):
            import torch
            if b.dtype != torch.float64 or not b.is_contiguous():
                raise TypeError("device right-hand side must be a contiguous float64 tensor")
            x, loc, bp = torch.empty_like(b), N.PSK_DEVICE, b
            torch_stream_ready(b, x)
        else:
            bp = np.ascontiguousarray(b, dtype=np.float64)
            x, loc = np.empty_like(bp), N.PSK_HOST
        fn = getattr(N.lib, self._entry)
        N.check(fn(dA.handle, ph, N.ptr(bp), N.ptr(x), ctypes.byref(ctl), ctypes.byref(res), N.ptr(hist), loc),
                self._entry)
        return self._to_status(res, x, hist[:res.hist_len])

    def _to_status(self, res, x, hist):
        normB = res.norm_b
        for k, nr in enumerate(hist):                        # reportIter replay (PCGSolver.py:126)
            self.reportIter(k, nr, normB)
        if res.status == N.PSK_CONVERGED:
            st = self.handleConvergence(res.iters - 1, x, res.resid, normB)
        elif res.status == N.PSK_BREAKDOWN:
            st = self.handleBreakdown(res.iters, res.msg.decode())
        elif res.status == N.PSK_MAXITER:
            st = self.handleMaxiter(res.iters, x, res.resid, normB)
        else:                                                # GMRES true residual miss (:167-174)
            st = SolveStatus(success=False, iters=res.iters, soln=x, resid=res.resid, msg=res.msg.decode())
        st.info = dict(status=N.STATUS_NAMES.get(res.status, str(res.status)), hist=np.array(hist),
                       loop_ms=res.loop_ms, spmv_ms=res.spmv_ms, spmv_launches=res.spmv_launches,
                       resid_recursive=res.resid_recursive, norm_b=normB)
        return st


def mvmult(A, x):
    """IterativeLinearSolver.py:94-106, on the device for sparse (and DeviceCSR) A."""
    if isinstance(A, DeviceCSR) or sp.issparse(A):
        return spmv(A, x)
    return spmv(sp.csr_matrix(np.asarray(A, dtype=np.float64)), x)
