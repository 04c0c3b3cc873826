"""The strip triangular-solve schedule (sptrsv_strip_kernel, ilu.hip, round 4): strips of the natural
index per workgroup, rows of a strip in steps of <= 64 independent rows, one row per lane, in-strip
dependencies from an LDS ring. Its per-row arithmetic is the grid / band kernels' (one fma chain over
the entries in stored order, then (b - acc) / d), not the sync-free family's lane partials + wave
total, so the bar against the sync-free schedule and against the host reference solve (SuperLU
ILU.solve / spsolve_triangular) is 1e-12 relative, as for every triangular chain, and
re-applies must be bitwise reproducible. The layout is planned for factors of more than 18432 rows
without a grid schedule (or with PSK_TRISOLVE_STRIP=1 at creation)."""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

pytestmark = pytest.mark.gpu

SCHED = {"syncfree": 0, "part": 4, "strip": 5}


@pytest.fixture(scope="module")
def psk():
    import pysolvers_amd
    return pysolvers_amd


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _set(h, which, sched):
    from pysolvers_amd import _native as N
    sc = ctypes.c_int32()
    N.check(N.lib.psk_prec_trisolve_schedule(h, which, -1 if sched is None else SCHED[sched], ctypes.byref(sc),
                                             None, None, None, None), "psk_prec_trisolve_schedule")
    return sc.value


@pytest.mark.parametrize("m", [192, 512, 1024])
def test_strip_schedule_ilut(psk, monkeypatch, m):
    """RightILUT of FD m^2 (the reference's spilu call, COLAMD order): the strip apply matches
    ILU.solve and the sync-free schedule to 1e-12 and is bitwise reproducible; mixed schedules
    (strip L, sync-free U and the reverse) too."""
    from oracle import fdlap
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    v = np.random.default_rng(m).standard_normal(A.shape[0])
    monkeypatch.setenv("PSK_TRISOLVE_STRIP", "1")
    M = psk.RightILUT().form(A)
    monkeypatch.delenv("PSK_TRISOLVE_STRIP")
    h = M.device_handle
    assert _set(h, 0, None) == 5 and _set(h, 1, None) == 5
    ref = M.ILU().solve(v)
    p = M.applyRight(v)
    assert _rel(p, ref) <= 1e-12
    assert np.array_equal(M.applyRight(v), p)        # re-apply: sentinel refill, fresh LDS ring
    _set(h, 1, "syncfree")
    assert _rel(M.applyRight(v), ref) <= 1e-12       # strip L, sync-free U
    _set(h, 0, "syncfree")
    q = M.applyRight(v)
    assert _rel(q, ref) <= 1e-12 and _rel(p, q) <= 1e-12
    _set(h, 1, "strip")                              # sync-free L, strip U
    assert _rel(M.applyRight(v), ref) <= 1e-12


def test_strip_schedule_random_long_rows(psk, monkeypatch):
    """Random unit-lower / upper factors with permuted input and output and rows of 300-900
    entries (steps then hold few rows: the chunk bound), n = 50000."""
    from pysolvers_amd.Linear import TriangularSolveChain
    n = 50000
    rng = np.random.default_rng(11)
    Lo = sp.tril(sp.random(n, n, density=6.0 / n, random_state=rng), k=-1).tolil()
    for r in rng.choice(np.arange(n // 2, n), 20, replace=False):
        cols = rng.choice(r, min(r, int(rng.integers(300, 900))), replace=False)
        Lo[r, cols] = rng.random(len(cols)) * 1e-3
    Lo = Lo.tocsr() * 0.1
    Up = sp.triu(sp.random(n, n, density=6.0 / n, random_state=rng), k=1).tocsr() * 0.1
    L = (Lo + sp.eye(n)).tocsr()
    U = (Up + sp.diags(1.0 + rng.random(n))).tocsr()
    gin, gout = rng.permutation(n), rng.permutation(n)
    v = rng.standard_normal(n)
    ref = spla.spsolve_triangular(U, spla.spsolve_triangular(L, v[gin], lower=True), lower=False)[gout]
    monkeypatch.setenv("PSK_TRISOLVE_STRIP", "1")
    M = TriangularSolveChain(n, L=L, l_unit=True, U=U, gather_in=gin, gather_out=gout)
    monkeypatch.delenv("PSK_TRISOLVE_STRIP")
    assert M.schedule("L")["schedule"] == "strip" and M.schedule("U")["schedule"] == "strip"
    out = M.apply(v)
    assert _rel(out, ref) <= 1e-12
    assert np.array_equal(M.apply(v), out)


def test_strip_gmres_ilut_matches_oracle(psk, monkeypatch):
    """GMRES(30) + RightILUT on FD 256^2 with both factors on the strip schedule, 60 steps (two
    restart cycles) vs the oracle GMRES(m) driven by the same SuperLU factors: residual history
    within 1e-10 ||b||, iterate within 1e-10 (the configs[2] test's bars)."""
    from oracle import fdlap, krylov
    from pysolvers_amd import CommonSolverArgs
    m = 256
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    b = A @ np.random.default_rng(12345).random(m * m)
    monkeypatch.setenv("PSK_TRISOLVE_STRIP", "1")
    M = psk.RightILUT().form(A)
    monkeypatch.delenv("PSK_TRISOLVE_STRIP")
    assert _set(M.device_handle, 0, None) == 5 and _set(M.device_handle, 1, None) == 5
    steps = 60
    ctl = CommonSolverArgs(maxiter=steps, tau=0.0, failOnMaxiter=False, showIters=False, showFinal=False)
    s = psk.GMRES(control=ctl, precond=psk.RightILUT(), restart=30).makeSolver()
    s.precond = M
    s.freezePrec()
    st = s.solve(A, b)
    ref = krylov.gmres_restarted(A, b, 30, maxiter=steps, tau=0.0, fail_on_maxiter=False, precond=M.ILU().solve)
    nb = np.linalg.norm(b)
    assert st.iters() == ref["iters"]
    assert np.max(np.abs(st.info["hist"] - ref["hist"])) / nb <= 1e-10
    assert np.linalg.norm(st.soln() - ref["soln"]) <= 1e-10 * np.linalg.norm(ref["soln"])
