"""Right-preconditioned GMRES: factory ``GMRES`` and ``GMRESSolver`` (GMRESSolver.py:27-180).

Arnoldi (MGS), Givens and the convergence test run on the GPU (``psk_gmres``).
``restart=0`` (default) is the reference's non-restarted method with Krylov
dimension ``maxiter``; ``restart=m`` gives GMRES(m), which the reference lacks.
The reference's two crashes are not reproduced: the
preconditioner is always formed (GMRESSolver.py:71 reads an unset attribute)
and reaching maxiter returns the handleMaxiter status instead of a NameError
(:180), with the current iterate as soln.
"""
from ..IterativeSolver import CommonSolverArgs
from .IterativeLinearSolver import IterativeLinearSolver, IterativeLinearSolverType
from .PreconditionerType import IdentityPreconditionerType


class GMRES(IterativeLinearSolverType):
    def __init__(self, control=CommonSolverArgs(), precond=IdentityPreconditionerType(), name='GMRES',
                 restart=0):
        super().__init__(control=control, precond=precond, name=name)
        self._restart = int(restart)

    def makeSolver(self, name=None):
        return GMRESSolver(self.control(), precond=self.precond(), name=self.name() if name is None else name,
                           restart=self._restart)


class GMRESSolver(IterativeLinearSolver):
    _entry = "psk_gmres"

    def __init__(self, control=CommonSolverArgs(), precond=IdentityPreconditionerType(), name='GMRES',
                 restart=0):
        super().__init__(control=control, precond=precond, name=name)
        self.restart = int(restart)

    def _restart(self):
        return self.restart

    def solve(self, A, b):
        return self._device_solve(A, b)
