"""BASELINE configs[2] and configs[4] exercised at their workload size on the device.

configs[2]: GMRES(30) + RightILUT on FDLaplacian2D. The reference's own ILUT (spilu drop_tol=1e-3,
fill_factor=15; ILUTPreconditioner.py:51-53) cannot be formed at 4096^2 by scipy's SuperLU
(SUPERLU_MALLOC fails, in the reference too), so the largest formable side, 2896, is the test size:
the first 60 Arnoldi steps (two GMRES(30) cycles, so the restart r = b - A x and a second cycle
from it are crossed at size) on the device vs the oracle GMRES(m) driven by the SAME SuperLU factors
(ILU.solve on the host, ILUTPreconditioner.py:77-78).

configs[4]: PCG + AMG(numIters=2, 5 levels) on -FDLaplacian2D 8192^2 (FDBratu2D.py:15 sign): the
hierarchy's level sizes, every device operator against the host scipy operators bit for bit, each
coarse operator against R_k (A_{k+1} P_k) recomputed on the host (MLHierarchy.py:54), a few PCG
iterations (run-to-run bitwise), the apply's linearity, and after 6 iterations the reported (recursive)
residual against the true residual of the returned x. At -FD 2048^2 (4.2M rows) one AMG apply and two PCG+AMG iterations
are compared with the oracle's V-cycle (oracle/amg.py) over the same hierarchy.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL_RESID = 1e-10


@pytest.fixture(scope="module")
def psk():
    import pysolvers_amd
    from pysolvers_amd import _native as N
    assert N.device_count() >= 1, "no GPU visible to libpsk"
    return pysolvers_amd


def _ctl(**kw):
    from pysolvers_amd import CommonSolverArgs
    kw.setdefault("showIters", False)
    kw.setdefault("showFinal", False)
    return CommonSolverArgs(**kw)


def _bitwise(A, B):
    A, B = A.tocsr(), B.tocsr()
    return (A.shape == B.shape and np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
            and np.array_equal(A.data.view(np.uint64), B.data.view(np.uint64)))


def test_configs2_gmres30_ilut_fd2896(psk):
    """configs[2] at FD 2896^2 (8.4M rows, L+U ~ 3.7e8 entries): 60 GMRES(30)+ILUT steps = two restart
    cycles (GMRESSolver.py:87-160 per cycle), residual history within 1e-10 ||b|| of the oracle's and
    the iterate within 1e-10 relative."""
    from oracle import fdlap, krylov
    m = 2896
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    b = A @ np.random.default_rng(12345).random(m * m)
    M = psk.RightILUT().form(A)                  # spilu on the host, factors uploaded once
    ilu = M.ILU()
    steps = 60
    ctl = _ctl(maxiter=steps, tau=0.0, failOnMaxiter=False)
    s = psk.GMRES(control=ctl, precond=psk.RightILUT(), restart=30).makeSolver()
    s.precond = M                                # the same factors, as a frozen preconditioner
    s.freezePrec()
    st = s.solve(A, b)
    ref = krylov.gmres_restarted(A, b, 30, maxiter=steps, tau=0.0, fail_on_maxiter=False, precond=ilu.solve)
    assert st.iters() == ref["iters"] == steps - 1 and st.success() and ref["success"]
    nb = np.linalg.norm(b)
    h = st.info["hist"]
    assert len(h) == len(ref["hist"]) == steps
    assert np.max(np.abs(h - ref["hist"])) / nb <= RTOL_RESID
    assert np.linalg.norm(st.soln() - ref["soln"]) <= 1e-10 * np.linalg.norm(ref["soln"])


LEVELS_8192 = [16642, 131423, 1243743, 11186176, 67108864]


def test_configs4_amg_hierarchy_and_pcg_fd8192(psk):
    """configs[4] at -FD 8192^2 (67M rows), 5 levels: level sizes, device operators == host scipy
    operators, coarse operators == R (A P) on the host, PCG+AMG iterations bitwise reproducible."""
    dA0 = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, 8192)
    A = -dA0.to_scipy()
    del dA0
    dA = psk.DeviceCSR.from_scipy(A)
    M = psk.AMG(numIters=2, numLevels=5).form(dA)
    assert M.levels() == LEVELS_8192
    mlh = M.mlh
    for k in range(4):
        assert _bitwise(M._A[k].to_scipy(), mlh.matrix(k)), k
        assert _bitwise(M._P[k].to_scipy(), mlh.update(k)), k
        assert _bitwise(M._R[k].to_scipy(), mlh.downdate(k)), k
        Ac = mlh.downdate(k) * (mlh.matrix(k + 1) * mlh.update(k))       # MLHierarchy.py:54
        assert _bitwise(Ac, mlh.matrix(k)), k
    assert _bitwise(dA.to_scipy(), A)
    b = A @ np.random.default_rng(12345).random(A.shape[0])
    ctl = _ctl(maxiter=3, tau=0.0, failOnMaxiter=False)
    s = psk.PCG(control=ctl, precond=psk.AMG(numIters=2, numLevels=5)).makeSolver()
    s.precond = M
    s.freezePrec()
    st1 = s.solve(dA, b)
    st2 = s.solve(dA, b)
    assert st1.iters() == st2.iters() == 3 and st1.success()
    assert np.array_equal(st1.info["hist"], st2.info["hist"]) and np.array_equal(st1.soln(), st2.soln())
    assert np.all(np.isfinite(st1.info["hist"])) and st1.info["hist"][-1] < np.linalg.norm(b)
    # full-size property past the oracle's reach: the recursive residual the loop reports (PCGSolver.py:122,
    # 125) and the true residual of the returned x agree within 1e-10 ||b|| after 6 PCG+AMG iterations
    ctl6 = _ctl(maxiter=6, tau=0.0, failOnMaxiter=False)
    s6 = psk.PCG(control=ctl6, precond=psk.AMG(numIters=2, numLevels=5)).makeSolver()
    s6.precond = M
    s6.freezePrec()
    st6 = s6.solve(dA, b)
    assert st6.iters() == 6 and np.array_equal(st6.info["hist"][:3], st1.info["hist"])
    r6 = b - psk.mvmult(dA, st6.soln())
    assert abs(np.linalg.norm(r6) - st6.info["hist"][-1]) <= RTOL_RESID * np.linalg.norm(b)
    # size-independent property at full size: the V-cycle apply (x = copy(v), VCycleSolver.py:69, then
    # cycles of smoothing / restriction / prolongation, no convergence snapshot for random v) is
    # linear in v, so M(u + 2 v) = M(u) + 2 M(v) up to rounding
    rng = np.random.default_rng(8192)
    u, v = rng.standard_normal(A.shape[0]), rng.standard_normal(A.shape[0])
    yu, yv, yuv = M.applyRight(u), M.applyRight(v), M.applyRight(u + 2.0 * v)
    assert np.all(np.isfinite(yuv))
    assert np.linalg.norm(yuv - (yu + 2.0 * yv)) <= 1e-10 * np.linalg.norm(yuv)
    # round 6: the fine level's Gauss-Seidel sweeps run two per launch (amg.hip gs_pair_kernel); at full size the
    # apply and the PCG+AMG trajectory equal the serialized sweeps' bit for bit (psk_lab_amg_gs_pair switches)
    import ctypes
    from pysolvers_amd import _native as N
    lab = N.load_lab()
    on, el = ctypes.c_int32(), ctypes.c_int32()
    N.check(lab.psk_lab_amg_gs_pair(M.device_handle, -1, ctypes.byref(on), ctypes.byref(el)), "gs_pair")
    assert (on.value, el.value) == (1, 1)
    N.check(lab.psk_lab_amg_gs_pair(M.device_handle, 0, None, None), "gs_pair off")
    try:
        yu_serial = M.applyRight(u)
        st_serial = s.solve(dA, b)
    finally:
        N.check(lab.psk_lab_amg_gs_pair(M.device_handle, 1, None, None), "gs_pair on")
    assert np.array_equal(yu_serial, yu)
    assert np.array_equal(st_serial.info["hist"], st1.info["hist"]) and np.array_equal(st_serial.soln(), st1.soln())


def test_configs4_amg_apply_and_pcg_vs_oracle_fd2048(psk):
    """-FD 2048^2 (4.2M rows), 5 levels: one AMG apply and two PCG+AMG iterations against the oracle's
    V-cycle over the same hierarchy (Gauss-Seidel by spsolve_triangular: the reference's spsolve of
    triu(A) takes 98 s per sweep at this size)."""
    from oracle import amg, fdlap, krylov
    m = 2048
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    M = psk.AMG(numIters=2, numLevels=5).form(A)
    mlh = M.mlh
    levels = ([mlh.matrix(k) for k in range(5)], [mlh.update(k) for k in range(4)],
              [mlh.downdate(k) for k in range(4)])
    ref = amg.AMGApply(A, num_iters=2, levels=levels, tri=True)
    v = np.random.default_rng(11).standard_normal(A.shape[0])
    y, yr = M.applyRight(v), ref(v)
    assert np.linalg.norm(y - yr) <= 1e-10 * np.linalg.norm(yr)
    b = A @ np.random.default_rng(12345).random(A.shape[0])
    ctl = _ctl(maxiter=2, tau=0.0, failOnMaxiter=False)
    s = psk.PCG(control=ctl, precond=psk.AMG(numIters=2, numLevels=5)).makeSolver()
    s.precond = M
    s.freezePrec()
    st = s.solve(A, b)
    ro = krylov.pcg(A, b, maxiter=2, tau=0.0, fail_on_maxiter=False, precond=ref)
    assert st.iters() == ro["iters"] == 2
    nb = np.linalg.norm(b)
    assert np.max(np.abs(st.info["hist"] - ro["hist"])) / nb <= RTOL_RESID
    assert np.linalg.norm(st.soln() - ro["soln"]) <= 1e-10 * np.linalg.norm(ro["soln"])
