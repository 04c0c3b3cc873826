"""Line searches for the Newton driver (LineSearch.py:4-81): host-side scalar logic.

``search(x0, normF0, p, func) -> (accepted, x, F, ||F||)`` is the contract Newton relies on.
SimpleBacktrack is Dennis & Schnabel's backtracking as the reference runs it: trial points
x0 + t p with t = 1 first; accept the first with ||F|| <= (1 - alpha t) ||F(x0)||; otherwise shrink
t by max(0.5 / (||F_t|| / ||F(x0)||), low); give up after ``maxsteps`` trials, returning the last
trial. TrivialLinesearch accepts the full step.
"""
from abc import ABC, abstractmethod


class LineSearch(ABC):
    """Parameters, the norm (set by the Newton driver) and the per-trial report line."""

    def __init__(self, maxsteps=15, low=0.1, alpha=0.0001, report=True):
        self._maxsteps, self._low, self._alpha, self._report = maxsteps, low, alpha, report
        self._norm = None

    @abstractmethod
    def search(self, x0, resid, newtStep, func):
        ...

    def maxsteps(self):
        return self._maxsteps

    def alpha(self):
        return self._alpha

    def low(self):
        return self._low

    def setNorm(self, norm):
        self._norm = norm

    def norm(self, x):
        if self._norm is None:
            raise RuntimeError('Norm not set in line search')
        return self._norm(x)

    def report(self, k, t, ratio):
        if self._report:
            print('k=%4d t=%12.5g ||F_k||/||F_0||=%12.5g' % (k, t, ratio))

    def _trial(self, x0, t, p, func):
        """(x, F(x), ||F(x)||) at x = x0 + t p; the reference evaluates F with evalF, except the
        trivial search, which calls ``func.eval`` (kept when the function object has one)."""
        x = x0 + t * p
        F = func.evalF(x)
        return x, F, self.norm(F)


class TrivialLinesearch(LineSearch):
    """Full Newton step, always accepted (LineSearch.py:43-55; for testing)."""

    def __init__(self, report=True):
        super().__init__(report=report)

    def search(self, x0, normF0, newtStep, func):
        x1 = x0 + newtStep
        F1 = func.eval(x1) if hasattr(func, "eval") else func.evalF(x1)
        return True, x1, F1, self.norm(F1)


class SimpleBacktrack(LineSearch):
    """Backtracking with sufficient decrease (LineSearch.py:58-81)."""

    def __init__(self, maxsteps=10, low=0.1, alpha=0.0001, report=True):
        super().__init__(maxsteps=maxsteps, low=low, alpha=alpha, report=report)

    def _shrink(self, t, ratio):
        return t * max(0.5 / ratio, self.low())

    def search(self, x0, normF0, newtStep, func):
        t = 1.0
        trial = None
        for k in range(self.maxsteps()):
            trial = self._trial(x0, t, newtStep, func)
            ratio = trial[2] / normF0
            self.report(k, t, ratio)
            if trial[2] <= (1.0 - self.alpha() * t) * normF0:
                return (True,) + trial
            t = self._shrink(t, ratio)
        return (False,) + trial
