#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run only in the build container, where the reference is mounted read-only at
/root/reference:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does
------------
* imports the reference package (krlong014/PySolvers) from /root/reference.  Two
  external modules the reference imports are absent from the image (PyTab,
  PyTimer); they only print indentation / timing, so minimal
  stand-ins are injected into ``sys.modules`` (nothing is written into the
  reference tree; bytecode writing is disabled);
* runs the reference solvers (PCG, patched GMRES), its FD generator, its mvmult
  and its Givens helpers on seeded inputs;
* runs the oracle restatement (oracle/) on the same inputs in the same process
  and ASSERTS bit-identity (iteration counts, residual histories, solutions);
* writes inputs + reference outputs as compressed .npz fixtures.  Fixtures are
  data only (matrices, vectors, scalars); no reference source is stored.

The GPU box never runs this file (it has no /root/reference).
"""
import contextlib
import hashlib
import io
import json
import os
import sys
import types

import numpy as np
import scipy.sparse as sp
from scipy.io import mmread

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)


def _install_standins():
    tab = types.ModuleType("PyTab")

    class Tab:                       # used only as an indentation prefix in prints
        def __str__(self):
            return ""

        def indent(self):
            pass

        def unindent(self):
            pass
    tab.Tab = Tab
    sys.modules["PyTab"] = tab
    tm = types.ModuleType("PyTimer")

    class Timer:                     # used only by SA-AMG setup timing
        def __init__(self, *a, **k):
            pass

        def start(self):
            pass

        def stop(self):
            pass

        @staticmethod
        def report():
            pass
    tm.Timer = Timer
    sys.modules["PyTimer"] = tm


_install_standins()
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(REF, "examples"))

from PySolvers import CommonSolverArgs                                   # noqa: E402
from PySolvers.Linear import PCG, GMRES, RightILUT, RightIC, AMG         # noqa: E402
from PySolvers.Linear.ClassicSmoothers import JacobiSmoother as RefJacobiSmoother   # noqa: E402
from PySolvers.Linear.SmoothedAggregation import SmoothedAggregationMLHierarchy     # noqa: E402
from PySolvers.Linear.PreconditionerType import PreconditionerType       # noqa: E402
from PySolvers.Linear.Preconditioner import GenericPreconditioner        # noqa: E402
from PySolvers.Linear.IterativeLinearSolver import mvmult as ref_mvmult  # noqa: E402
from PySolvers.Linear import Givens as ref_givens                        # noqa: E402
from FDLaplacian2D import FDLaplacian2D as ref_fd2d                      # noqa: E402

from oracle import amg, krylov, fdlap, newton                             # noqa: E402
from PySolvers.Nonlinear import NewtonSolver                             # noqa: E402
from FDBratu2D import FDBratu2D as RefBratu                              # noqa: E402

# AMG preconditioner variants of the golden cases: name -> (numIters, numLevels, smoother)
AMG_VARIANTS = {"amg": (2, 2, "gs"), "amg_jacobi": (2, 2, "jacobi"), "amg3": (2, 3, "gs")}


class _JacobiPrec(GenericPreconditioner):
    """Jacobi through the reference's own plugin API (Preconditioner.py:20-36)."""

    def __init__(self, A):
        self.DInv = np.reciprocal(A.diagonal())

    def apply(self, vec):
        return np.multiply(self.DInv, vec)


class _Jacobi(PreconditionerType):
    def form(self, A):
        return _JacobiPrec(A)


def _pname(jac):
    """Case preconditioner flag -> name: False/True (identity/Jacobi) or a name such as "ilut"."""
    return jac if isinstance(jac, str) else ("jacobi" if jac else "identity")


def _oracle_prec(A, jac):
    name = _pname(jac)
    if name in AMG_VARIANTS:
        it, lv, sm = AMG_VARIANTS[name]
        return amg.AMGApply(sp.csr_matrix(A), num_iters=it, num_levels=lv, smoother=sm)
    return {"identity": lambda: krylov.identity_apply, "jacobi": lambda: krylov.jacobi_form(A),
            "ilut": lambda: krylov.ilut_form(A), "ic": lambda: krylov.ic_form(A)}[name]()


def _ref_prec_type(name):
    if name in AMG_VARIANTS:
        it, lv, sm = AMG_VARIANTS[name]
        return AMG(numIters=it, numLevels=lv, **({"smoother": RefJacobiSmoother} if sm == "jacobi" else {}))
    return {"identity": None, "jacobi": _Jacobi(), "ilut": RightILUT(), "ic": RightIC()}[name]


def _run_ref(kind, A, b, maxiter, tau, fail_on_maxiter=True, jacobi=False):
    ctl = CommonSolverArgs(maxiter=maxiter, tau=tau, failOnMaxiter=fail_on_maxiter,
                           showIters=False, showFinal=False)
    pt = _ref_prec_type(_pname(jacobi))
    if kind == "pcg":
        st = (PCG(control=ctl, precond=pt) if pt else PCG(control=ctl)).makeSolver()
    else:
        st = (GMRES(control=ctl, precond=pt) if pt else GMRES(control=ctl)).makeSolver()
        st.precond = None          # GMRESSolver.py:71 reads an attribute it never sets
    hist = []
    st.reportIter = lambda it, nr, n0: hist.append(float(nr))
    with contextlib.redirect_stdout(io.StringIO()):
        res = st.solve(A, b)
    return res, np.array(hist)


def _check_same(tag, res, hist, orc):
    assert res.iters() == orc["iters"], (tag, res.iters(), orc["iters"])
    assert bool(res.success()) == bool(orc["success"]), tag
    assert np.array_equal(hist, orc["hist"]), tag
    if res.soln() is not None:
        assert np.array_equal(res.soln(), orc["soln"]), tag
    if res.resid() is not None:
        assert float(res.resid()) == float(orc["resid"]), tag


def sensitivity(kind, A, b, maxiter, tau, fom, jac, hist_ref, soln_ref, seeds=8):
    """How far the reference path itself moves when every dot/norm is perturbed by <= 1 ulp.

    Runs the oracle (bit-identical to the reference) with np.dot / npla.norm results multiplied by
    (1 + e), e in {-2^-52, 0, 2^-52}, for `seeds` random draws. Returns the max over seeds of
    max_k |hist_k - hist_ref_k| / ||b|| and of ||x - x_ref|| / ||x_ref||, plus whether every
    perturbed run kept the reference's iteration count. This is the floor any re-implementation
    with a different (even exact) dot rounding can be held to.
    """
    import math
    import numpy.linalg as npla_
    od, on = krylov.np.dot, krylov.npla.norm
    nb = np.linalg.norm(b)
    dh, dx, same = 0.0, 0.0, True
    for seed in range(seeds):
        rng = np.random.default_rng(1000 + seed)

        def pdot(a, c):
            return od(a, c) * (1.0 + rng.choice([-1.0, 0.0, 1.0]) * 2.0 ** -52)
        krylov.np.dot = pdot
        krylov.npla.norm = lambda v: math.sqrt(pdot(v, v))
        try:
            prec = _oracle_prec(A, jac)
            fn = krylov.pcg if kind == "pcg" else krylov.gmres
            st = fn(A, b, maxiter=maxiter, tau=tau, fail_on_maxiter=fom, precond=prec)
        finally:
            krylov.np.dot, krylov.npla.norm = od, on
        h = st["hist"]
        m = min(len(h), len(hist_ref))
        same &= len(h) == len(hist_ref)
        if m:
            dh = max(dh, float(np.max(np.abs(h[:m] - hist_ref[:m])) / nb))
        if soln_ref is not None and st["soln"] is not None and np.linalg.norm(soln_ref) > 0:
            dx = max(dx, float(np.linalg.norm(st["soln"] - soln_ref) / np.linalg.norm(soln_ref)))
    return dict(hist_over_normb=dh, x_rel=dx, iters_stable=bool(same))


def _csr_arrays(A):
    A = A.tocsr()
    return dict(indptr=A.indptr.astype(np.int32), indices=A.indices.astype(np.int32),
                data=A.data.astype(np.float64), n=np.int64(A.shape[0]))


def _sha(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _dh(lev):
    return mmread(os.path.join(REF, "TestMatrices", "DH-Matrix-%d.mtx" % lev)).tocsr()


def main():
    out = {}
    manifest = {}

    # --- FD generator: full arrays for small m, hashes for larger m -----------------
    fd_small = {}
    for m in (1, 2, 3, 5, 16):
        A = ref_fd2d(-1.0, 1.0, m)
        ip, ix, dt = fdlap.fd_laplacian_2d_arrays(-1.0, 1.0, m)
        assert np.array_equal(A.indptr, ip) and np.array_equal(A.indices, ix) \
            and np.array_equal(A.data, dt), m
        fd_small["m%d_indptr" % m] = A.indptr.astype(np.int32)
        fd_small["m%d_indices" % m] = A.indices.astype(np.int32)
        fd_small["m%d_data" % m] = A.data
    hashes = {}
    for m in (64, 128, 300):
        A = ref_fd2d(-1.0, 1.0, m)
        ip, ix, dt = fdlap.fd_laplacian_2d_arrays(-1.0, 1.0, m)
        assert np.array_equal(A.indptr, ip) and np.array_equal(A.indices, ix) \
            and np.array_equal(A.data, dt), m
        hashes[str(m)] = dict(sha256=_sha(A.indptr.astype(np.int32), A.indices.astype(np.int32),
                                          A.data), nnz=int(A.nnz))
    np.savez_compressed(os.path.join(HERE, "fd_generator.npz"), **fd_small)
    manifest["fd_generator_sha256"] = hashes
    print("fd generator: ok")

    # --- SpMV golden (stored-order, non-sorted FD rows; and a DH matrix) -------------
    A = ref_fd2d(-1.0, 1.0, 64)
    x = np.random.default_rng(7).random(A.shape[0])
    y = ref_mvmult(A, x)
    A8 = _dh(8)
    x8 = np.random.default_rng(8).random(A8.shape[0])
    y8 = ref_mvmult(A8, x8)
    np.savez_compressed(os.path.join(HERE, "spmv.npz"),
                        fd64_x=x, fd64_y=y, dh8_x=x8, dh8_y=y8,
                        **{"fd64_" + k: v for k, v in _csr_arrays(A).items()},
                        **{"dh8_" + k: v for k, v in _csr_arrays(A8).items()})
    print("spmv: ok")

    # --- Givens self-test (Givens.py:36-120) ------------------------------------------
    H, g = krylov.givens_selftest_matrix()
    Hr, gr = H.copy(), g.copy()
    n_, m_ = Hr.shape
    CS = np.zeros([m_, 2])
    for i in range(m_):
        for j in range(i):
            ref_givens.applyGivensInPlace(Hr[:, i], CS[j, 0], CS[j, 1], j)
        CS[i, :] = ref_givens.findGivensCoefficients(Hr[:, i], i)
        ref_givens.applyGivensInPlace(Hr[:, i], CS[i, 0], CS[i, 1], i)
        ref_givens.applyGivensInPlace(gr, CS[i, 0], CS[i, 1], i)
    yr = np.linalg.solve(Hr[0:m_, :], gr[0:m_])
    Ho, go, CSo, yo = krylov.givens_triangularize(H, g)
    assert np.array_equal(Hr, Ho) and np.array_equal(gr, go) and np.array_equal(yr, yo)
    np.savez_compressed(os.path.join(HERE, "givens.npz"), H=H, g=g, H_rot=Hr, g_rot=gr, CS=CS, y=yr)
    print("givens: ok")

    # --- AMG hierarchies and one apply each (SmoothedAggregation.py, VCycleManager.py) -----
    amg_fix = {}
    amg_index = []
    for name, A in (("dh8", _dh(8)), ("dh10", _dh(10)), ("negfd16", -ref_fd2d(-1.0, 1.0, 16)),
                    ("fd16", ref_fd2d(-1.0, 1.0, 16)), ("negfd32", -ref_fd2d(-1.0, 1.0, 32))):
        A = sp.csr_matrix(A)
        for L in (2, 3):
            with contextlib.redirect_stdout(io.StringIO()):
                h = SmoothedAggregationMLHierarchy(A, numLevels=L)
            ops, Ps, Rs = amg.hierarchy(A, L)
            key = "%s_L%d" % (name, L)
            for k in range(L):
                Mr, Mo = h.matrix(k).tocsr(), ops[k]
                assert np.array_equal(Mr.indptr, Mo.indptr) and np.array_equal(Mr.indices, Mo.indices) \
                    and np.array_equal(Mr.data, Mo.data), (key, k)
                for tag, M in (("A%d" % k, Mr),) + ((("P%d" % k, h.update(k).tocsr()), ("R%d" % k, h.downdate(k).tocsr()))
                                                       if k < L - 1 else ()):
                    amg_fix["%s_%s_indptr" % (key, tag)] = M.indptr.astype(np.int32)
                    amg_fix["%s_%s_indices" % (key, tag)] = M.indices.astype(np.int32)
                    amg_fix["%s_%s_data" % (key, tag)] = M.data
                    amg_fix["%s_%s_shape" % (key, tag)] = np.array(M.shape, dtype=np.int64)
                if k < L - 1:
                    for Mr_, Mo_ in ((h.update(k).tocsr(), Ps[k]), (h.downdate(k).tocsr(), Rs[k])):
                        assert np.array_equal(Mr_.indptr, Mo_.indptr) and np.array_equal(Mr_.indices, Mo_.indices) \
                            and np.array_equal(Mr_.data, Mo_.data), (key, k)
            v = np.random.default_rng(7).standard_normal(A.shape[0])
            amg_fix[key + "_v"] = v
            for sm, cls in (("gs", None), ("jacobi", RefJacobiSmoother)):
                with contextlib.redirect_stdout(io.StringIO()):
                    M = (AMG(numIters=2, numLevels=L, smoother=cls) if cls else AMG(numIters=2, numLevels=L)).form(A)
                    y = M.apply(v)
                yo = amg.AMGApply(A, num_iters=2, num_levels=L, smoother=sm)(v)
                assert np.array_equal(y, yo), (key, sm)
                amg_fix["%s_apply_%s" % (key, sm)] = y
            amg_index.append(dict(key=key, levels=[int(o.shape[0]) for o in ops]))
    np.savez_compressed(os.path.join(HERE, "amg_hierarchy.npz"), **amg_fix)
    manifest["amg_hierarchy"] = amg_index
    print("amg hierarchy: ok", [d["key"] for d in amg_index])

    # --- Solver cases ------------------------------------------------------------------
    cases = []
    for lev in (8, 10, 12, 15):
        cases.append(("pcg", "dh%d" % lev, _dh(lev), 2000, 1e-8, True, False))
    for lev in (8, 10):
        cases.append(("pcg", "dh%d" % lev, _dh(lev), 2000, 1e-8, True, True))
    for m in (16, 64, 128):
        cases.append(("pcg", "fd%d" % m, ref_fd2d(-1.0, 1.0, m), 4000, 1e-8, True, True))
    cases.append(("pcg", "fd32", ref_fd2d(-1.0, 1.0, 32), 4000, 1e-8, True, False))
    # maxiter edge cases (IterativeSolver.py:115-129 / PCGSolver.py:129-131)
    cases.append(("pcg", "dh8_maxiter10_fail", _dh(8), 10, 1e-8, True, False))
    cases.append(("pcg", "dh8_maxiter10_nofail", _dh(8), 10, 1e-8, False, False))
    cases.append(("pcg", "dh8_maxiter1_fail", _dh(8), 1, 1e-8, True, False))
    cases.append(("pcg", "fd16_tau0_nofail", ref_fd2d(-1.0, 1.0, 16), 25, 0.0, False, True))
    # GMRES (patched, non-restarted): maxiter large enough to converge (GMRESSolver.py:180)
    for lev in (8, 10):
        cases.append(("gmres", "dh%d" % lev, _dh(lev), 300, 1e-8, True, False))
    cases.append(("gmres", "dh8", _dh(8), 300, 1e-8, True, True))
    cases.append(("gmres", "fd16", ref_fd2d(-1.0, 1.0, 16), 300, 1e-8, True, False))
    cases.append(("gmres", "fd16", ref_fd2d(-1.0, 1.0, 16), 300, 1e-8, True, True))
    cases.append(("gmres", "fd32", ref_fd2d(-1.0, 1.0, 32), 300, 1e-10, True, True))
    # GMRES + RightILUT (examples/GMRESExample_ILUT.py plumbing, configs[2] at small sizes)
    for lev in (8, 10):
        cases.append(("gmres", "dh%d" % lev, _dh(lev), 100, 1e-8, True, "ilut"))
    for m in (32, 64):
        cases.append(("gmres", "fd%d" % m, ref_fd2d(-1.0, 1.0, m), 100, 1e-8, True, "ilut"))
    cases.append(("pcg", "dh10", _dh(10), 300, 1e-8, True, "ilut"))
    # PCG + RightIC (examples/PCGExample_IC.py plumbing)
    for lev in (8, 10, 12):
        cases.append(("pcg", "dh%d" % lev, _dh(lev), 300, 1e-8, True, "ic"))
    cases.append(("pcg", "negfd32", -ref_fd2d(-1.0, 1.0, 32), 300, 1e-8, True, "ic"))   # IC needs SPD
    # PCG/GMRES + AMG (examples/PCGExample_AMG.py: AMG(numIters=2); config 5 at small sizes)
    for lev in (8, 10, 12):
        cases.append(("pcg", "dh%d" % lev, _dh(lev), 100, 1e-8, True, "amg"))
    cases.append(("pcg", "dh10", _dh(10), 100, 1e-8, True, "amg_jacobi"))
    cases.append(("pcg", "dh10", _dh(10), 100, 1e-8, True, "amg3"))
    cases.append(("gmres", "dh8", _dh(8), 100, 1e-8, True, "amg"))
    # -FD2D (FDBratu2D.py:15 sign): PCG+AMG does not converge: 10 iterations, no fail
    cases.append(("pcg", "negfd32_maxiter10_nofail", -ref_fd2d(-1.0, 1.0, 32), 10, 1e-8, False, "amg"))

    index = []
    for kind, name, A, maxiter, tau, fom, jac in cases:
        b, xex = fdlap.manufactured_rhs(A, 12345)
        # b from the reference's own mvmult must equal the oracle's
        assert np.array_equal(b, ref_mvmult(A, xex))
        res, hist = _run_ref(kind, A, b, maxiter, tau, fom, jac)
        prec = _oracle_prec(A, jac)
        fn = krylov.pcg if kind == "pcg" else krylov.gmres
        orc = fn(A, b, maxiter=maxiter, tau=tau, fail_on_maxiter=fom, precond=prec)
        tag = "%s_%s_%s" % (kind, name, _pname(jac))
        _check_same(tag, res, hist, orc)
        fname = tag + ".npz"
        payload = dict(b=b, x_exact=xex, hist=hist, maxiter=np.int64(maxiter), tau=np.float64(tau),
                       fail_on_maxiter=np.int64(fom), jacobi=np.int64(_pname(jac) == "jacobi"),
                       precond=np.array(_pname(jac)),
                       iters=np.int64(res.iters()), success=np.int64(bool(res.success())),
                       resid=np.float64(res.resid() if res.resid() is not None else np.nan),
                       soln=res.soln() if res.soln() is not None else np.zeros(0),
                       **_csr_arrays(A))
        np.savez_compressed(os.path.join(HERE, fname), **payload)
        index.append(dict(file=fname, kind=kind, matrix=name, n=int(A.shape[0]), nnz=int(A.nnz),
                          maxiter=maxiter, tau=tau, fail_on_maxiter=fom, jacobi=_pname(jac) == "jacobi",
                          precond=_pname(jac),
                          iters=int(res.iters()), success=bool(res.success()),
                          resid=None if res.resid() is None else float(res.resid()),
                          final_ratio=float(hist[-1] / np.linalg.norm(b)) if len(hist) else None,
                          sensitivity=sensitivity(kind, A, b, maxiter, tau, fom, jac, hist, res.soln())))
        print("%-40s iters=%5d success=%s sens=%s" % (tag, res.iters(), res.success(), index[-1]["sensitivity"]))

    # --- Newton + PCG on FD-Bratu (examples/FDBratu2D.py:33-48), the caller of the hot path ------
    newton_index = []
    for m, pname in ((32, "ic"), (32, "amg5"), (64, "ic")):
        func = RefBratu(m=m)
        pt = RightIC() if pname == "ic" else AMG(numIters=5)
        ctl = CommonSolverArgs(tau=1.0e-12, maxiter=10, showIters=False, showFinal=False)
        lin_ctl = CommonSolverArgs(showIters=False, showFinal=False)
        ns = NewtonSolver(control=ctl, solver=PCG(control=lin_ctl, precond=pt), fixLinTol=False, minLinTol=1.0e-6,
                          freezePrec=True)
        hist, lin = [], []
        ns.reportIter = lambda it, nr, n0: hist.append(float(nr))
        inner = ns.solver.solve

        def counting_solve(A_, b_, inner=inner, lin=lin):
            st_ = inner(A_, b_)
            lin.append(st_.iters())
            return st_
        ns.solver.solve = counting_solve
        with contextlib.redirect_stdout(io.StringIO()):
            res = ns.solve(func, func.initialU())
        fp = (lambda J: krylov.ic_form(J)) if pname == "ic" else (lambda J: amg.AMGApply(J, num_iters=5))
        orc = newton.newton(newton.Bratu2D(m=m), np.ones(m * m), fp, maxiter=10, tau=1e-12, min_lin_tol=1e-6)
        assert orc["iters"] == res.iters() and bool(orc["success"]) == bool(res.success()), (m, pname)
        assert np.array_equal(orc["hist"], np.array(hist)) and orc["linear_iters"] == lin, (m, pname)
        if res.soln() is not None:
            assert np.array_equal(orc["soln"], res.soln())
        tag = "newton_bratu%d_%s" % (m, pname)
        np.savez_compressed(os.path.join(HERE, tag + ".npz"), hist=np.array(hist), linear_iters=np.array(lin),
                            soln=res.soln() if res.soln() is not None else np.zeros(0))
        newton_index.append(dict(file=tag + ".npz", m=m, precond=pname, iters=int(res.iters()),
                                 success=bool(res.success()), msg=res.msg(), linear_iters=[int(v) for v in lin]))
        print("%-28s iters=%d success=%s linear=%s msg=%s" % (tag, res.iters(), res.success(), lin, res.msg()))
    manifest["newton"] = newton_index

    # b = 0 (PCGSolver.py:86-88, GMRESSolver.py:66-68): iters=1, x=0
    A = _dh(8)
    for kind in ("pcg", "gmres"):
        res, hist = _run_ref(kind, A, np.zeros(A.shape[0]), 50, 1e-8)
        assert res.iters() == 1 and res.success() and not np.any(res.soln())
    manifest["zero_rhs"] = dict(iters=1, success=True, resid=0)

    manifest["cases"] = index
    manifest["generator"] = "tests/golden/make_golden.py"
    manifest["numpy"] = np.__version__
    import scipy
    manifest["scipy"] = scipy.__version__
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(index), "solver fixtures")


if __name__ == "__main__":
    main()
