"""Control object, status object and the iterative-solver base class.

Same public surface as the reference's PySolvers/IterativeSolver.py,
PySolvers/SolveStatus.py and PySolvers/NamedObject.py, so callers (drivers,
Newton) are unchanged:

* ``CommonSolverArgs(maxiter=100, failOnMaxiter=True, tau=1e-8, norm=npla.norm,
  showIters=True, showFinal=True, interval=1)``      (IterativeSolver.py:42-57)
* ``SolveStatus(success, soln, resid, iters, msg)`` with the accessors
  ``success() soln() resid() iters() msg()``          (SolveStatus.py:12-56)
* ``IterativeSolver``: maxiter/failOnMaxiter/tau/setTolerance/norm and the
  report* printers                                     (IterativeSolver.py:62-155)

``norm`` may be any callable, as in the reference: the device loops use the
Euclidean norm (``npla.norm``, the default) in-loop; another norm makes PCG run
host-driven over the same device kernels (the norm of r is the caller's code,
PCGSolver.py:86,125) and GMRES apply it to b and to the final true residual
(GMRESSolver.py:66,164; its Arnoldi norms are npla.norm in the reference too).
"""
import numpy.linalg as npla


class NamedObject:
    """Object with a name (NamedObject.py:2-11)."""

    def __init__(self, name=''):
        self._name = name

    def name(self):
        return self._name


class SolveStatus:
    """Outcome of a solve (SolveStatus.py:8-56)."""

    __slots__ = ("_success", "_soln", "_resid", "_iters", "_msg", "info")

    def __init__(self, success, soln, resid, iters, msg=None):
        self._success = success
        self._soln = soln
        self._resid = resid
        self._iters = iters
        self._msg = msg
        self.info = {}          # device-side extras: status code, timings, history

    def success(self):
        return self._success

    def soln(self):
        return self._soln

    def resid(self):
        return self._resid

    def iters(self):
        return self._iters

    def msg(self):
        return self._msg

    def __str__(self):
        return 'SolverState(success={}, resid={}, iters={})'.format(
            self._success, self._resid, self._iters)


class CommonSolverArgs:
    """Typical control parameters of an iterative solver (IterativeSolver.py:25-57)."""

    def __init__(self, maxiter=100, failOnMaxiter=True, tau=1.0e-8, norm=npla.norm,
                 showIters=True, showFinal=True, interval=1):
        self.maxiter = maxiter
        self.failOnMaxiter = failOnMaxiter
        self.tau = tau
        self.norm = norm
        self.showIters = showIters
        self.showFinal = showFinal
        self.interval = interval


class IterativeSolver(NamedObject):
    """Shared control/reporting logic (IterativeSolver.py:62-155)."""

    def __init__(self, control, name=''):
        super().__init__(name)
        self._control = control

    def maxiter(self):
        return self._control.maxiter

    def failOnMaxiter(self):
        return self._control.failOnMaxiter

    def tau(self):
        return self._control.tau

    def setTolerance(self, tau):
        self._control.tau = tau

    def norm(self, x):
        return self._control.norm(x)

    def _custom_norm(self):
        """True when CommonSolverArgs.norm is not numpy.linalg.norm (IterativeSolver.py:86-88)."""
        return self._control.norm is not npla.norm

    # --- printing, same text as the reference ---------------------------------------------
    def reportIter(self, iter, normR, normR0):
        c = self._control
        if c.showIters and (iter % c.interval) == 0:
            print('%s iter=%7d ||r||=%12.5g ||r||/r0=%12.5g' % (self.name(), iter, normR, normR / normR0))

    def reportSuccess(self, iter, normR, normB):
        if self._control.showFinal:
            rel = normR / normB if normR != 0 else normR
            print('%s solve succeeded: iters=%7d, ||r||/r0=%12.5g' % (self.name(), iter, rel))

    def reportBreakdown(self, msg=''):
        if self._control.showFinal:
            print('%s solve broke down: %s' % (self.name(), msg))

    def reportFailure(self, iter, normR, normB):
        if self._control.showFinal:
            print('%s solve FAILED: iters=%7d, ||r||/r0=%12.5g' % (self.name(), iter, normR / normB))

    # --- status construction (IterativeSolver.py:101-129) ------------------------------------
    def handleConvergence(self, iter, x, normR, normB):
        self.reportSuccess(iter + 1, normR, normB)
        return SolveStatus(success=True, iters=iter + 1, soln=x, resid=normR)

    def handleBreakdown(self, iter, msg):
        self.reportBreakdown(msg=msg)
        return SolveStatus(success=False, iters=iter, soln=None, resid=None, msg=msg)

    def handleMaxiter(self, iter, x, normR, normB):
        if self.failOnMaxiter():
            self.reportFailure(iter, normR, normB)
            return SolveStatus(success=False, iters=iter, soln=x, resid=normR, msg='failure to converge')
        self.reportSuccess(iter + 1, normR, normB)
        return SolveStatus(success=True, iters=iter, soln=x, resid=normR)
