"""``DefaultDirect``: the direct linear solver factory NewtonSolver defaults to
(DefaultDirectSolver.py:22-74, Newton.py:13).

The reference calls ``spla.spsolve(A, b)`` (SuperLU factor + solve, every call) for a sparse A and
``npla.solve`` for a dense one, and turns any exception into a failed SolveStatus. Here the
factorisation is the one ``spsolve`` performs — computed on the host by SuperLU, as the AMG coarse
level does (AMGPreconditioner.coarse_factor: spsolve's COLAMD factors of a CSR matrix) — and the
two triangular solves run on the device (TriangularSolveChain, the same sync-free / band / LDS
kernels as ILUT and the coarse solve). A dense A is handed over as CSR. The factors of the last
matrix are kept, so repeated solves with the same A object (a frozen Newton Jacobian) factor once.
Status conventions as the reference: SolveStatus(True, x, None, None, '<name> solve succeeded') or
SolveStatus(False, None, None, None, '<name> solve failed: <error>').
"""
import numpy as np
import scipy.sparse as sp

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
        self._src = None
        self._op = None

    def _operator(self, A):
        from .AMGPreconditioner import coarse_solver
        if self._op is not None and self._src is A:
            return self._op
        if isinstance(A, DeviceCSR):
            A = A.to_scipy()
        elif not sp.issparse(A):
            if not isinstance(A, np.ndarray):
                raise TypeError('not numpy or scipy')
            A = sp.csr_matrix(A)
        self._op, _ = coarse_solver(sp.csr_matrix(A))
        self._src = A
        return self._op

    def solve(self, A, b):
        n, nc = A.shape
        assert n == nc                               # DefaultDirectSolver.py:56-58
        assert n == len(b)
        if not (sp.issparse(A) or isinstance(A, (np.ndarray, DeviceCSR))):
            return SolveStatus(False, None, None, None, 'Input to solver [%s] not numpy or scipy' % self.name())
        try:
            x = self._operator(A).apply(b)
            return SolveStatus(True, x, None, None, '%s solve succeeded' % self.name())
        except Exception as ex:                      # :72-74
            return SolveStatus(False, None, None, None, '{} solve failed: {}'.format(self.name(), ex))
