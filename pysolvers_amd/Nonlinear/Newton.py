"""Inexact Newton driver over the device linear solvers (the caller of the hot path, Newton.py:10-101).

Function and Jacobian evaluation are the caller's host code (``func.evalF`` / ``func.evalJ``), as
in the reference; every Newton step's linear solve J p = -F is one libpsk solve (device PCG/GMRES,
or the device-applied direct solve of ``DefaultDirect``). Semantics kept from the reference:

* convergence test before each step: ||F_i|| <= tau ||F_0|| + tau (:54);
* linear tolerance per step: ``minLinTol`` if ``fixLinTol`` else max(tolFudge ||F_i|| / ||F_0||,
  minLinTol) (:62-73), set only on iterative linear solvers;
* with ``freezePrec`` the preconditioner formed for the first Jacobian is reused for every later
  one (PreconditionerFreeze.py:15-21; the reference never unfreezes);
* a failed linear solve or line search ends the solve through handleBreakdown (:79-82, :95-97);
  maxiter through handleMaxiter(maxiter, ...) (:101);
* the unconditional 'freeze prec for solver=' line the reference prints (:38) is printed too.
"""
from ..IterativeSolver import CommonSolverArgs, IterativeSolver
from ..Linear.DirectSolver import DefaultDirect
from ..Linear.IterativeLinearSolver import IterativeLinearSolver
from .LineSearch import SimpleBacktrack
from .PreconditionerFreeze import PreconditionerFreeze


class NewtonSolver(IterativeSolver):
    def __init__(self, control=CommonSolverArgs(), solver=DefaultDirect(), linesearch=SimpleBacktrack(),
                 fixLinTol=False, tolFudge=0.1, minLinTol=1.0e-10, freezePrec=True, name='Newton'):
        super().__init__(control, name=name)
        self.solver = solver.makeSolver()
        self.linesearch = linesearch
        self.fixLinTol = fixLinTol
        self.tolFudge = tolFudge
        self.minLinTol = minLinTol
        self.freezePrec = freezePrec
        self.linear_iters = []          # iterations of each step's linear solve (diagnostics)

    def _linear_tolerance(self, normF, normF0):
        """Tolerance handed to an iterative step solver (:62-73)."""
        if self.fixLinTol:
            return self.minLinTol
        return max(self.tolFudge * normF / normF0, self.minLinTol)

    def _converged(self, normF, normF0):
        return normF <= normF0 * self.tau() + self.tau()

    def _step(self, J, F, normF, normF0):
        """Newton direction p with J p = -F, or (None, message) when the linear solve failed."""
        if isinstance(self.solver, IterativeLinearSolver):
            self.solver.setTolerance(self._linear_tolerance(normF, normF0))
        status = self.solver.solve(J, -F)
        self.linear_iters.append(status.iters())
        if status.success():
            return status.soln(), None
        return None, 'solve for Newton step failed with msg={}'.format(status.msg())

    def solve(self, func, xInit):
        x = xInit.copy()
        F = func.evalF(x)
        print('freeze prec for solver=', self.freezePrec)
        PreconditionerFreeze(self.solver, self.freezePrec)
        self.linesearch.setNorm(self.norm)
        normF0 = self.norm(F)
        normF = normF0
        self.linear_iters = []
        i = 0
        while i < self.maxiter():
            self.reportIter(i, normF, normF0)
            if self._converged(normF, normF0):
                return self.handleConvergence(i, x, normF, normF0)
            p, why = self._step(func.evalJ(x), F, normF, normF0)
            if p is None:
                return self.handleBreakdown(i, why)
            accepted, x, F, normF = self.linesearch.search(x, normF, p, func)
            if not accepted:
                return self.handleBreakdown(i, msg='Line search failed')
            i += 1
        return self.handleMaxiter(self.maxiter(), x, normF, normF0)
