"""Newton's method with a device Krylov solver for the steps (Newton.py:10-101).

The loop is host logic (function and Jacobian evaluation are the caller's numpy code, as in the
reference); each step's J p = -F solve is one device PCG/GMRES call with the adaptive tolerance
max(tolFudge ||F||/||F_0||, minLinTol) (:62-73) and, with freezePrec, the preconditioner formed on
the first Jacobian reused for every later step (:38-39, PreconditionerFreeze).
"""
from ..IterativeSolver import CommonSolverArgs, IterativeSolver
from ..Linear.IterativeLinearSolver import IterativeLinearSolver
from .LineSearch import SimpleBacktrack
from .PreconditionerFreeze import PreconditionerFreeze


class NewtonSolver(IterativeSolver):
    def __init__(self, control=CommonSolverArgs(), solver=None, linesearch=SimpleBacktrack(), fixLinTol=False,
                 tolFudge=0.1, minLinTol=1.0e-10, freezePrec=True, name='Newton'):
        super().__init__(control, name=name)
        if solver is None:
            # the reference's default is DefaultDirect() (a SuperLU wrapper, outside this build's hot path)
            raise TypeError("NewtonSolver: pass solver=PCG(...) or GMRES(...) (the direct-solver default "
                            "DefaultDirect is not part of this build)")
        self.solver = solver.makeSolver()
        self.linesearch = linesearch
        self.fixLinTol = fixLinTol
        self.tolFudge = tolFudge
        self.minLinTol = minLinTol
        self.freezePrec = freezePrec
        self.linear_iters = []          # iterations of each step's linear solve (diagnostics)

    def solve(self, func, xInit):
        xCur = xInit.copy()
        FCur = func.evalF(xCur)
        print('freeze prec for solver=', self.freezePrec)
        PreconditionerFreeze(self.solver, self.freezePrec)
        self.linesearch.setNorm(self.norm)
        r0 = self.norm(FCur)
        normFCur = r0
        self.linear_iters = []
        for i in range(self.maxiter()):
            self.reportIter(i, normFCur, r0)
            if normFCur <= r0 * self.tau() + self.tau():                       # :54
                return self.handleConvergence(i, xCur, normFCur, r0)
            J = func.evalJ(xCur)
            if isinstance(self.solver, IterativeLinearSolver):
                tau_lin = self.minLinTol if self.fixLinTol else max(self.tolFudge * normFCur / r0, self.minLinTol)
                self.solver.setTolerance(tau_lin)
            status = self.solver.solve(J, -FCur)
            self.linear_iters.append(status.iters())
            if not status.success():
                return self.handleBreakdown(i, 'solve for Newton step failed with msg={}'.format(status.msg()))
            p = status.soln()
            (success, xCur, FCur, normFCur) = self.linesearch.search(xCur, normFCur, p, func)
            if not success:
                return self.handleBreakdown(i, msg='Line search failed')
        return self.handleMaxiter(self.maxiter(), xCur, normFCur, r0)
