"""``DefaultDirect``: the direct linear solver factory NewtonSolver defaults to
(DefaultDirectSolver.py:22-74, Newton.py:13).

The reference calls ``spla.spsolve(A, b)`` (SuperLU factor + solve, every call) for a sparse A and
``npla.solve`` for a dense one, and turns any exception into a failed SolveStatus. Here the
factorisation is the one ``spsolve`` performs — computed on the host by SuperLU, as the AMG coarse
level does (AMGPreconditioner.coarse_factor: spsolve's COLAMD factors of a CSR matrix) — and the
two triangular solves run on the device (TriangularSolveChain, the same sync-free / band / LDS
kernels as ILUT and the coarse solve). A dense A is handed over as CSR. The factors of the last
matrix are kept and reused only while its CONTENTS (indptr, indices, data) are unchanged, so a
frozen Newton Jacobian factors once and a Jacobian updated in place is refactored, as spsolve would.
Status conventions as the reference: SolveStatus(True, x, None, None, '<name> solve succeeded') or
SolveStatus(False, None, None, None, '<name> solve failed: <error>'). An exactly singular sparse
matrix behaves as spsolve does there: a MatrixRankWarning and an all-NaN solution with a SUCCESS
status (spsolve does not raise; the reference only fails on an exception). A DENSE ndarray goes to
npla.solve in the reference, whose LinAlgError on an exactly singular matrix becomes
SolveStatus(False, None, None, None, '<name> solve failed: Singular matrix'); here the same status is
returned when the SuperLU factorisation of that matrix finds it exactly singular (make_direct.py pins
both conventions; LAPACK's partial pivoting and SuperLU's ordering could disagree on a matrix that
is singular only in one of the two pivot orders — no fixture has one).
"""
import warnings

import numpy as np
import scipy.sparse as sp
from scipy.sparse.linalg import MatrixRankWarning

from ..IterativeSolver import SolveStatus
from .DeviceMatrix import DeviceCSR
from .LinearSolver import LinearSolver, LinearSolverType


class DefaultDirect(LinearSolverType):
    def __init__(self, name='Default direct'):
        super().__init__(name=name)

    def makeSolver(self, name=None):
        return DefaultDirectSolver(name=self.name() if name is None else name)


class DefaultDirectSolver(LinearSolver):
    def __init__(self, name='Default direct'):
        super().__init__(name=name)
        self._key = None     # (indptr, indices, data) copies of the factored matrix
        self._op = None      # device solve operator, or None when that matrix is exactly singular

    def _operator(self, A):
        """(operator, singular) for A; refactored whenever A's contents differ from the cached ones."""
        from .AMGPreconditioner import coarse_solver
        if isinstance(A, DeviceCSR):
            A = A.to_scipy()
        elif not sp.issparse(A):
            if not isinstance(A, np.ndarray):
                raise TypeError('not numpy or scipy')
            A = sp.csr_matrix(A)
        A = sp.csr_matrix(A)
        if self._key is not None and all(np.array_equal(a, b) for a, b in zip(self._key, (A.indptr, A.indices, A.data))):
            return self._op, self._op is None
        self._key = (A.indptr.copy(), A.indices.copy(), A.data.copy())
        try:
            self._op, _ = coarse_solver(A)
        except RuntimeError as ex:
            if 'exactly singular' not in str(ex):
                self._key = None
                raise
            self._op = None
        return self._op, self._op is None

    def solve(self, A, b):
        n, nc = A.shape
        assert n == nc                               # DefaultDirectSolver.py:56-58
        assert n == len(b)
        if not (sp.issparse(A) or isinstance(A, (np.ndarray, DeviceCSR))):
            return SolveStatus(False, None, None, None, 'Input to solver [%s] not numpy or scipy' % self.name())
        dense = isinstance(A, np.ndarray)
        try:
            op, singular = self._operator(A)
            if singular and dense:                   # npla.solve (:64-65) raises LinAlgError -> failure
                return SolveStatus(False, None, None, None, '%s solve failed: Singular matrix' % self.name())
            if singular:                             # spsolve: warning + NaN solution, no exception
                warnings.warn("Matrix is exactly singular", MatrixRankWarning, stacklevel=2)
                x = np.full(n, np.nan)
            else:
                x = op.apply(b)
            return SolveStatus(True, x, None, None, '%s solve succeeded' % self.name())
        except Exception as ex:                      # :72-74
            return SolveStatus(False, None, None, None, '{} solve failed: {}'.format(self.name(), ex))
