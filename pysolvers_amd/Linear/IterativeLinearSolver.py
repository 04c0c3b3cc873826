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
    # PCGSolver.solve prints 'prec frozen = ...' and 'building prec' on every solve with b != 0
    # (PCGSolver.py:91,93); PCGSolver sets this (class attribute: a driver may switch it off)
    _echo_setup = False

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
        custom = self._custom_norm()
        normb_caller = 0.0
        if custom:
            normb_caller = float(self.norm(_host_copy(b)))     # self.norm(b)  PCGSolver.py:86, GMRESSolver.py:66
            zero_b = normb_caller == 0.0
        else:
            zero_b = _is_zero_norm(b, n)                       # the default norm: ||b|| == 0 iff b.b == 0
        if zero_b:                                             # :87-88 / :67-68: x = 0, before the
            x0 = DeviceVector(n) if isinstance(b, DeviceVector) else np.zeros(n)   # preconditioner is formed
            if isinstance(x0, DeviceVector):
                x0.zero()
            return self.handleConvergence(0, _like(b, x0), 0, 0)
        dA = self._device_matrix(A)
        echo = self._echo_setup
        if echo:                                            # PCGSolver.py:91 (unconditional in the reference)
            print('prec frozen = ', self.precFrozen())
        if self.precond is None or not self.precFrozen():   # PCGSolver.py:92-94
            if echo:
                print('building prec')                      # :93
            self.precond = self.precondType().form(dA)
        if custom and self._entry == "psk_pcg":
            return self._host_norm_pcg(dA, b, normb_caller)
        kind = getattr(self.precond, "device_kind", None)
        if kind is None:
            raise TypeError("%s: preconditioner %r has no device implementation; available: "
                            "IdentityPreconditionerType, JacobiPreconditionerType, RightILUT, RightIC, AMG"
                            % (self.name(), type(self.precond).__name__))
        ph = None if kind == N.PSK_PREC_IDENTITY else self.precond.device_handle

        maxiter = int(self.maxiter())
        ctl = N.PskCtl(maxiter=maxiter, tau=float(self.tau()), fail_on_maxiter=int(bool(self.failOnMaxiter())),
                       restart=int(self._restart()), check_every=0, time_kernels=int(bool(self.time_kernels)),
                       norm_b=normb_caller)
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
        if custom and res.exit in (N.PSK_EXIT_TOLERANCE, N.PSK_EXIT_ARNOLDI_BREAKDOWN):
            # GMRES stopped on its recursive residual: the true-residual test in the caller's norm
            # (GMRESSolver.py:163-174): resid = b - A x on the device, its norm by the caller's code
            rt = _host_copy(b) - _host_copy(spmv(dA, x))
            nrt = float(self.norm(rt))
            ok = nrt <= self.tau() * normb_caller
            res.resid = nrt
            res.status = N.PSK_CONVERGED if ok else N.PSK_TRUE_RESID_FAIL
            res.success = int(ok)
            res.msg = b"" if ok else (
                "GMRES failure: true residual %12.5g did not meet tolerance tau=%12.5g. Recursive residual "
                "was %12.5g." % (nrt, self.tau(), res.resid_recursive)).encode()
        return self._to_status(res, x, hist[:res.hist_len])

    # -----------------------------------------------------------------------------------------
    def _host_norm_pcg(self, dA, b, normB):
        """PCG (PCGSolver.py:97-142) with a caller-supplied norm: the loop is driven from the host
        over the device kernels (SpMV, dot, AXPY-type updates, preconditioner apply), because the
        reference evaluates self.norm(r) every iteration (:125) and that is the caller's host code;
        r is copied to the host for it. Same operation order and status conventions as psk_pcg."""
        n = dA.n
        prec = self.precond

        def result(x):                             # the kind of vector the caller passed (as psk_pcg)
            return x if isinstance(b, DeviceVector) else _like(b, x.numpy())

        def dot(u, v):
            out = ctypes.c_double()
            N.check(N.lib.psk_dot(n, u._p, v._p, N.PSK_DEVICE, ctypes.byref(out)), "psk_dot")
            return out.value

        def axpy(alpha, v, y):                     # y = y + alpha*v, two roundings (numpy)
            N.check(N.lib.psk_axpy(n, float(alpha), v._p, y._p, N.PSK_DEVICE), "psk_axpy")

        def copy(v):
            y = DeviceVector(n)
            y.zero()
            axpy(1.0, v, y)
            return y

        def apply(v):                              # precond.applyRight, never aliasing its input
            if getattr(prec, "device_kind", None) == N.PSK_PREC_IDENTITY:
                return copy(v)
            out = prec.applyRight(v)
            return copy(out) if out is v else out

        r = DeviceVector.from_numpy(_host_copy(b))                    # r = copy(b)  :97
        p = apply(r)                                                  # :98
        u = copy(p)                                                   # :99
        x = DeviceVector(n)
        x.zero()                                                      # :100
        uDotR = dot(u, r)                                             # :102
        if uDotR == 0.0:                                              # :104-105
            return self.handleBreakdown(0, 'breakdown dot(u,r)==0')
        k, normR = -1, None
        hist = []
        for k in range(self.maxiter()):                               # :109
            Ap = spmv(dA, p)                                          # :111
            pTAp = dot(p, Ap)                                         # :113
            if pTAp == 0.0:                                           # :114-115
                return self.handleBreakdown(k, 'breakdown dot(p, Ap)==0')
            alpha = uDotR / pTAp                                      # :118
            axpy(alpha, p, x)                                         # x = x + alpha*p  :121
            axpy(-alpha, Ap, r)                                       # r = r - alpha*Ap  :122
            u = apply(r)                                              # :123
            normR = float(self.norm(r.numpy()))                       # :125
            hist.append(normR)
            self.reportIter(k, normR, normB)                          # :126
            if normR <= self.tau() * normB or (not self.failOnMaxiter() and k == self.maxiter() - 1):
                st = self.handleConvergence(k, result(x), normR, normB)   # :129-131
                st.info = dict(status="converged", hist=np.array(hist), norm_b=normB, host_driven=True)
                return st
            newUDotR = dot(u, r)                                      # :134
            beta = newUDotR / uDotR                                   # :135
            uDotR = newUDotR                                          # :136
            axpy(beta, p, u)                                          # p = u + beta*p  :138
            p = u
        st = self.handleMaxiter(max(k, 0), result(x), normR, normB)   # :142
        st.info = dict(status="maxiter", hist=np.array(hist), norm_b=normB, host_driven=True)
        return st


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


def _like(b, x):
    """x (a host ndarray, or a DeviceVector when b is one) as the kind of vector b is: a CUDA tensor
    on b's device for a tensor b, else unchanged."""
    if is_device_vector(b) and not isinstance(x, DeviceVector):
        import torch
        return torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=b.device)
    return x


def _is_zero_norm(b, n):
    """||b|| == 0 (npla.norm(b) = sqrt(b.b), PCGSolver.py:86): the reference returns before its
    setup prints then. One dot over b (host numpy, or psk_nrm2 for a device vector)."""
    if isinstance(b, DeviceVector) or is_device_vector(b):
        out = ctypes.c_double()
        p = b._p if isinstance(b, DeviceVector) else N.ptr(b)
        if not isinstance(b, DeviceVector):
            torch_stream_ready(b)
        N.check(N.lib.psk_nrm2(n, p, N.PSK_DEVICE, ctypes.byref(out)), "psk_nrm2")
        return out.value == 0.0
    v = np.ascontiguousarray(b, dtype=np.float64)
    return float(np.dot(v, v)) == 0.0


def _host_copy(v):
    """A host ndarray of a vector given as ndarray, DeviceVector or CUDA tensor."""
    if isinstance(v, DeviceVector):
        return v.numpy()
    if is_device_vector(v):
        return v.detach().cpu().numpy()
    return np.asarray(v, dtype=np.float64)


def mvmult(A, x):
    """IterativeLinearSolver.py:94-106, on the device for sparse (and DeviceCSR) A. A dense ndarray A
    (the reference's `np.dot(A, x)`, :105-106, a BLAS dgemv) goes through CSR here: its row sums run in
    stored order, which rounds differently from dgemv's blocked order by a few ulps — dense-A results
    match the reference to rounding, not bit for bit (pinned by the reference's own dense PCG/GMRES runs,
    tests/golden/make_dense.py, at the solver cases' bars)."""
    if isinstance(A, DeviceCSR) or sp.issparse(A):
        return spmv(A, x)
    return spmv(sp.csr_matrix(np.asarray(A, dtype=np.float64)), x)
