"""CPU restatement of the reference's Newton caller and its FD-Bratu test problem (TEST INFRASTRUCTURE).

Only tests/ and the golden generator import this module.

* NewtonSolver.solve (Nonlinear/Newton.py:29-101) with SimpleBacktrack (LineSearch.py:58-81),
  driving the oracle PCG (oracle/krylov.py) with a frozen preconditioner (PreconditionerFreeze.py)
* FDBratu2D (examples/FDBratu2D.py:10-29): F(u) = A u - alpha exp(-u), J(u) = A + diag(alpha exp(-u)),
  A = -FDLaplacian2D(-1, 1, m)
"""
import numpy as np
import scipy.sparse.linalg as spla
import numpy.linalg as npla

from . import fdlap, krylov


class Bratu2D:
    def __init__(self, m=4, alpha=0.5):
        self.m = m
        self.alpha = alpha
        self.A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)

    def initialU(self):
        return np.ones(self.m * self.m)

    def evalF(self, u):
        return self.A * u - self.alpha * np.exp(-u)

    def evalJ(self, u):
        J = self.A.copy()
        g = self.alpha * np.exp(-u)
        d = J.diagonal()
        J.setdiag(d + g)
        return J


def simple_backtrack(x0, normF0, p, func, maxsteps=10, low=0.1, alpha=0.0001):
    t = 1.0
    for _ in range(maxsteps):
        x_k = x0 + t * p
        F_k = func.evalF(x_k)
        normF_k = npla.norm(F_k)
        ratio = normF_k / normF0
        if normF_k <= (1.0 - alpha * t) * normF0:
            return True, x_k, F_k, normF_k
        factor = 0.5 / ratio
        if factor < low:
            factor = low
        t = t * factor
    return False, x_k, F_k, normF_k


def newton(func, x0, form_prec, maxiter=10, tau=1e-12, tol_fudge=0.1, min_lin_tol=1e-6, lin_maxiter=100,
           direct=False):
    """Returns dict(success, iters, soln, resid, msg, hist, linear_iters). form_prec(J) -> apply;
    formed once on the first Jacobian (freezePrec=True). direct=True: the steps are the default
    DefaultDirect solves, spla.spsolve(J, -F) (DefaultDirectSolver.py:61-70, Newton.py:13)."""
    x = x0.copy()
    F = func.evalF(x)
    r0 = npla.norm(F)
    nF = r0
    hist, lin = [], []
    prec = None
    for i in range(maxiter):
        hist.append(nF)
        if nF <= r0 * tau + tau:
            return dict(success=True, iters=i + 1, soln=x, resid=nF, msg=None, hist=np.array(hist), linear_iters=lin)
        J = func.evalJ(x)
        if direct:
            lin.append(None)
            ok, x, F, nF = simple_backtrack(x, nF, spla.spsolve(J, -F), func)
            if not ok:
                return dict(success=False, iters=i, soln=None, resid=None, msg='Line search failed',
                            hist=np.array(hist), linear_iters=lin)
            continue
        tl = max(tol_fudge * nF / r0, min_lin_tol)
        if prec is None:
            prec = form_prec(J)
        st = krylov.pcg(J, -F, maxiter=lin_maxiter, tau=tl, fail_on_maxiter=True, precond=prec)
        lin.append(st["iters"])
        if not st["success"]:
            return dict(success=False, iters=i, soln=None, resid=None, hist=np.array(hist), linear_iters=lin,
                        msg='solve for Newton step failed with msg={}'.format(st["msg"]))
        ok, x, F, nF = simple_backtrack(x, nF, st["soln"], func)
        if not ok:
            return dict(success=False, iters=i, soln=None, resid=None, msg='Line search failed',
                        hist=np.array(hist), linear_iters=lin)
    return dict(success=False, iters=maxiter, soln=x, resid=nF, msg='failure to converge', hist=np.array(hist),
                linear_iters=lin)
