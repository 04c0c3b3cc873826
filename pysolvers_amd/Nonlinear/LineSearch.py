"""Line searches for Newton's method (LineSearch.py:4-81): host-side scalar logic."""
from abc import ABC, abstractmethod


class LineSearch(ABC):
    def __init__(self, maxsteps=15, low=0.1, alpha=0.0001, report=True):
        self._maxsteps = maxsteps
        self._alpha = alpha
        self._report = report
        self._low = low
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


class TrivialLinesearch(LineSearch):
    """Accepts the full step (:43-55). The reference calls ``func.eval``; functions here provide
    ``evalF`` (as every reference example does), which is used when ``eval`` is absent."""

    def __init__(self, report=True):
        super().__init__(report=report)

    def search(self, x0, normF0, newtStep, func):
        x1 = x0 + newtStep
        F1 = func.eval(x1) if hasattr(func, "eval") else func.evalF(x1)
        return (True, x1, F1, self.norm(F1))


class SimpleBacktrack(LineSearch):
    """Dennis & Schnabel backtracking (:58-81): t = 1, accept when ||F(x0 + t p)|| <= (1 - alpha t)
    ||F(x0)||, else t *= max(0.5 / ratio, low)."""

    def __init__(self, maxsteps=10, low=0.1, alpha=0.0001, report=True):
        super().__init__(maxsteps=maxsteps, low=low, alpha=alpha, report=report)

    def search(self, x0, normF0, newtStep, func):
        t = 1.0
        for k in range(self.maxsteps()):
            x_k = x0 + t * newtStep
            F_k = func.evalF(x_k)
            normF_k = self.norm(F_k)
            ratio = normF_k / normF0
            self.report(k, t, ratio)
            if normF_k <= (1.0 - self.alpha() * t) * normF0:
                return (True, x_k, F_k, normF_k)
            factor = 0.5 / ratio
            if factor < self.low():
                factor = self.low()
            t = t * factor
        return (False, x_k, F_k, normF_k)
