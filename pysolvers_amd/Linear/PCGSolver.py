"""Preconditioned CG: factory ``PCG`` and solver ``PCGSolver`` (PCGSolver.py:25-142).

``PCG(control, precond, name).makeSolver().solve(A, b)`` runs the whole CG loop
(SpMV, dots, updates, preconditioner apply, convergence test) on the GPU via
``psk_pcg``; results follow the reference's SolveStatus conventions
(iters=k+1 on convergence, k on maxiter failure, breakdown -> soln=None).
"""
from ..IterativeSolver import CommonSolverArgs
from .IterativeLinearSolver import IterativeLinearSolver, IterativeLinearSolverType
from .PreconditionerType import IdentityPreconditionerType


class PCG(IterativeLinearSolverType):
    def __init__(self, control=CommonSolverArgs(), precond=IdentityPreconditionerType(), name='PCG'):
        super().__init__(control=control, precond=precond, name=name)

    def makeSolver(self, name=None):
        return PCGSolver(self.control(), precond=self.precond(), name=self.name() if name is None else name)


class PCGSolver(IterativeLinearSolver):
    _entry = "psk_pcg"
    _echo_setup = True     # the reference's two setup prints (PCGSolver.py:91,93)

    def __init__(self, control=CommonSolverArgs(), precond=IdentityPreconditionerType(), name='PCG'):
        super().__init__(control=control, precond=precond, name=name)

    def solve(self, A, b):
        return self._device_solve(A, b)
