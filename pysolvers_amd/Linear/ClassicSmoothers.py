"""Relaxation smoothers of the AMG V-cycle (ClassicSmoothers.py:1-36), on the GPU.

Both of the reference's smoothers are a sweep x <- x + S^-1 (f - A x):
* JacobiSmoother      S^-1 r = DInv * r, DInv = reciprocal(diag A)      (:5-14)
* GaussSeidelSmoother S^-1 r = spsolve(triu(A), r)                      (:28-36)
Each class builds that S^-1 as a device operator (``.operator``); the V-cycle itself runs inside
libpsk (psk_prec_create_amg). ``apply(f, x, nu)`` keeps the reference's host-callable contract.
"""
import numpy as np
import scipy.sparse as sp

from .DeviceMatrix import DeviceCSR, spmv
from .Preconditioner import JacobiPreconditioner
from .TriangularSolve import TriangularSolveChain


def _host(A):
    return A.to_scipy() if isinstance(A, DeviceCSR) else sp.csr_matrix(A)


class _Smoother:
    def __init__(self, A, device_A=None):
        self.A = A
        self._dA = device_A if device_A is not None else (A if isinstance(A, DeviceCSR) else DeviceCSR.from_scipy(A))

    def apply(self, f, x, nu):
        """nu sweeps from x (host arrays): r = f - A*x; x = x + S^-1 r."""
        x = np.asarray(x, dtype=np.float64)
        for _ in range(nu):
            r = np.asarray(f, dtype=np.float64) - spmv(self._dA, x)
            x = x + self.operator.apply(r)
        return x


class JacobiSmoother(_Smoother):
    def __init__(self, A, device_A=None):
        super().__init__(A, device_A)
        self.operator = JacobiPreconditioner(self._dA)


class GaussSeidelSmoother(_Smoother):
    def __init__(self, A, device_A=None):
        super().__init__(A, device_A)
        self.U = sp.triu(_host(A)).tocsr()              # :33
        self.operator = TriangularSolveChain(self.U.shape[0], U=self.U, u_unit=False)
