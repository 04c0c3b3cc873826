"""RightIC (ICPreconditioner.py:20-63): incomplete Cholesky from SuperLU's ILU, applied on the GPU.

``form(A)`` repeats the reference's setup on the host with the same third-party calls
(spilu with ColPerm NATURAL and no pivoting, Lt = diag(1/sqrt(diag U)) U, L = Lt^T, :45-56);
``applyRight`` (:58-63: spsolve_triangular(L, v, lower) then spsolve_triangular(Lt, u, upper))
runs as one device triangular-solve chain (TriangularSolve.py).
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from .DeviceMatrix import DeviceCSR
from .Preconditioner import RightPreconditioner
from .PreconditionerType import PreconditionerType
from .TriangularSolve import TriangularSolveChain


class RightIC(PreconditionerType):
    def __init__(self, drop_tol=0.001, fill_factor=15):
        self.drop_tol = drop_tol
        self.fill_factor = fill_factor

    def form(self, A):
        return ICRightPreconditioner(A, drop_tol=self.drop_tol, fill_factor=self.fill_factor)


class ICRightPreconditioner(TriangularSolveChain, RightPreconditioner):
    """Incomplete Cholesky applied from the right; applyLeft is the identity (Preconditioner.py:49-56)."""

    def __init__(self, A, drop_tol=0.001, fill_factor=15):
        Ah = A.to_scipy() if isinstance(A, DeviceCSR) else A
        ILU = spla.spilu(Ah.tocsc(), drop_tol=drop_tol, fill_factor=fill_factor, diag_pivot_thresh=0.0,
                         options={'ColPerm': 'NATURAL'})
        n = Ah.shape[0]
        diagScale = np.reciprocal(np.sqrt(ILU.U.diagonal()))
        DInv = sp.dia_matrix((diagScale, [0]), shape=(n, n))
        Lt = DInv * ILU.U
        del ILU
        self._L = Lt.transpose().tocsr()
        self._Lt = Lt.tocsr()
        super().__init__(n, L=self._L, l_unit=False, U=self._Lt, u_unit=False)

    def applyRight(self, vec):
        return self._device_apply(vec)

    def applyLeft(self, vec):
        return vec
