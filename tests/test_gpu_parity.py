"""Parity of the HIP engine (through the C ABI) with the oracle and the reference's golden vectors.

Bars (BASELINE.json north_star): SpMV, the FD generator, the Jacobi diagonal and
the elementwise updates are bit-exact; solver iteration counts are identical and
residuals agree to 1e-10 relative.

"Residuals" are the relative residuals ||r_k||/||b|| the reference reports
(IterativeSolver.reportIter prints ||r||/r0): every history entry must agree to
RTOL_RESID = 1e-10 of ||b||. The device's dot products are rounded differently
from OpenBLAS (any re-implementation's are), so for the few ill-conditioned
trajectories where the REFERENCE ITSELF moves by more than that under 1-ulp
perturbations of its dots (measured per case by tests/golden/make_golden.py,
`sensitivity` in manifest.json; DH-10 identity PCG: 2.3e-10), the bar is
10x that measured sensitivity instead.
"""
import ctypes
import hashlib

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import (case_precond, dense_cases, golden_matrix, load_golden, manifest, oracle_prec, product_prec_type,
                      restarted_cases, solver_cases)

pytestmark = pytest.mark.gpu

RTOL_RESID = 1e-10        # north_star: residuals within 1e-10 relative


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


# ---------------------------------------------------------------------------------------------
# bit-exact kernels

@pytest.mark.parametrize("tag", ["fd64", "dh8"])
def test_spmv_bitwise_golden(psk, tag):
    d = load_golden("spmv.npz")
    A = golden_matrix(d, tag + "_")
    y = psk.mvmult(A, d[tag + "_x"])
    assert np.array_equal(y, d[tag + "_y"])


def _ragged_matrix(rng, n, long_rows=(), empty_rows=()):
    rows, cols = [], []
    for i in range(n):
        if i in empty_rows:
            continue
        k = 3000 if i in long_rows else int(rng.integers(1, 9))
        c = rng.choice(n, size=min(k, n), replace=False)
        rows += [i] * len(c)
        cols += list(c)
    vals = rng.standard_normal(len(rows))
    A = sp.coo_matrix((vals, (rows, cols)), shape=(n, n)).tocsr()
    # shuffle each row's stored order: the kernel must follow stored order, not column order
    for i in range(n):
        s, e = A.indptr[i], A.indptr[i + 1]
        p = rng.permutation(e - s)
        A.indices[s:e] = A.indices[s:e][p]
        A.data[s:e] = A.data[s:e][p]
    A.has_sorted_indices = False
    return A


@pytest.mark.parametrize("n,long_rows,empty_rows", [
    (1, (), ()), (7, (), (3,)), (257, (), (0, 256)), (5000, (17, 4096), (5, 6, 7)), (70001, (300,), (69999,)),
])
def test_spmv_bitwise_ragged(psk, n, long_rows, empty_rows):
    rng = np.random.default_rng(n)
    A = _ragged_matrix(rng, n, long_rows, empty_rows)
    x = rng.standard_normal(n)
    assert np.array_equal(psk.mvmult(A, x), A @ x)


def test_spmv_empty_matrix(psk):
    A = sp.csr_matrix((4, 4))
    assert np.array_equal(psk.mvmult(A, np.ones(4)), np.zeros(4))


@pytest.mark.parametrize("m", [1, 2, 3, 5, 16, 64, 300])
def test_fd_generator_device_bitwise(psk, m):
    from oracle import fdlap
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    A = dA.to_scipy()
    ip, ix, dt = fdlap.fd_laplacian_2d_arrays(-1.0, 1.0, m)
    assert np.array_equal(A.indptr, ip) and np.array_equal(A.indices, ix) and np.array_equal(A.data, dt)
    if str(m) in manifest()["fd_generator_sha256"]:
        h = hashlib.sha256()
        for a in (A.indptr, A.indices, A.data):
            h.update(np.ascontiguousarray(a).tobytes())
        assert h.hexdigest() == manifest()["fd_generator_sha256"][str(m)]["sha256"]


def test_jacobi_bitwise(psk):
    d = load_golden("spmv.npz")
    for tag in ("fd64", "dh8"):
        A = golden_matrix(d, tag + "_")
        M = psk.JacobiPreconditionerType().form(A)
        v = d[tag + "_x"]
        assert np.array_equal(M.applyRight(v), np.multiply(np.reciprocal(A.diagonal()), v))


def test_blas1(psk):
    from pysolvers_amd import _native as N
    rng = np.random.default_rng(3)
    for n in (1, 511, 512, 513, 100003):
        x, y = rng.standard_normal(n), rng.standard_normal(n)
        out = ctypes.c_double()
        N.check(N.lib.psk_dot(n, N.ptr(x), N.ptr(y), N.PSK_HOST, ctypes.byref(out)), "dot")
        assert abs(out.value - np.dot(x, y)) <= 1e-13 * np.abs(x) @ np.abs(y)
        N.check(N.lib.psk_nrm2(n, N.ptr(x), N.PSK_HOST, ctypes.byref(out)), "nrm2")
        assert abs(out.value - np.linalg.norm(x)) <= 1e-14 * np.linalg.norm(x)
        yy = y.copy()
        N.check(N.lib.psk_axpy(n, 0.37, N.ptr(x), N.ptr(yy), N.PSK_HOST), "axpy")
        assert np.array_equal(yy, y + 0.37 * x)      # two roundings, as numpy


# ---------------------------------------------------------------------------------------------
# solvers vs the reference's golden runs

def tolerances(case):
    sens = case.get("sensitivity") or {}
    th = max(RTOL_RESID, 10.0 * sens.get("hist_over_normb", 0.0))
    tx = max(1e-10, 10.0 * sens.get("x_rel", 0.0))
    return th, tx


def _check_against_golden(st, d, case):
    assert st.iters() == case["iters"], (st.iters(), case["iters"])
    assert bool(st.success()) == case["success"]
    th, tx = tolerances(case)
    h_ref = d["hist"]
    h = st.info["hist"]
    nb = np.linalg.norm(d["b"])
    assert len(h) == len(h_ref)
    if len(h):
        dev = np.max(np.abs(h - h_ref)) / nb
        assert dev <= th, ("relative residual history deviates", dev, th)
    if case["resid"] is not None:
        assert abs(st.resid() - case["resid"]) / nb <= th
    if d["soln"].size:
        err = np.linalg.norm(st.soln() - d["soln"]) / np.linalg.norm(d["soln"])
        assert err <= tx, ("solution deviates", err, tx)


@pytest.mark.parametrize("case", solver_cases(), ids=lambda c: c["file"][:-4])
def test_solver_matches_reference(psk, case):
    d = load_golden(case["file"])
    A = golden_matrix(d)
    ctl = _ctl(maxiter=case["maxiter"], tau=case["tau"], failOnMaxiter=bool(case["fail_on_maxiter"]))
    pt = product_prec_type(psk, case_precond(case))
    factory = psk.PCG if case["kind"] == "pcg" else psk.GMRES
    st = factory(control=ctl, precond=pt).makeSolver().solve(A, d["b"])
    _check_against_golden(st, d, case)


@pytest.mark.parametrize("case", dense_cases(), ids=lambda c: c["file"][:-4])
def test_dense_solver_matches_reference(psk, case):
    """A dense ndarray A (the reference's np.dot, IterativeLinearSolver.py:105-106 — a BLAS dgemv) runs on the
    device as CSR with stored-order row sums: the reference's own dense runs (tests/golden/make_dense.py) pin it
    with the solver cases' bars — identical iteration counts, residual history and solution within 1e-10 (or 10x
    the reference's own 1-ulp sensitivity)."""
    d = load_golden(case["file"])
    ctl = _ctl(maxiter=case["maxiter"], tau=case["tau"], failOnMaxiter=bool(case["fail_on_maxiter"]))
    pt = product_prec_type(psk, case_precond(case))
    factory = psk.PCG if case["kind"] == "pcg" else psk.GMRES
    A = d["A"]
    assert isinstance(A, np.ndarray)
    st = factory(control=ctl, precond=pt).makeSolver().solve(A, d["b"])
    _check_against_golden(st, d, case)


@pytest.mark.parametrize("kind", ["pcg", "gmres"])
def test_zero_rhs(psk, kind):
    d = load_golden("pcg_dh8_identity.npz")
    A = golden_matrix(d)
    f = psk.PCG if kind == "pcg" else psk.GMRES
    st = f(control=_ctl(maxiter=50)).makeSolver().solve(A, np.zeros(A.shape[0]))
    assert st.success() and st.iters() == 1 and not np.any(st.soln())
    # PCGSolver.py:86-88 / GMRESSolver.py:66-68 return before the preconditioner is formed
    s = f(control=_ctl(maxiter=50), precond=psk.Jacobi()).makeSolver()
    st = s.solve(A, psk.DeviceVector.from_numpy(np.zeros(A.shape[0])))
    assert st.success() and st.iters() == 1 and not np.any(st.soln().numpy()) and s.precond is None


def test_pcg_breakdown_zero_matrix(psk):
    # pTAp == 0 at k=0 -> handleBreakdown(0, ...) (PCGSolver.py:114-115): soln None, iters 0
    A = sp.csr_matrix((5, 5))
    st = psk.PCG(control=_ctl(maxiter=10)).makeSolver().solve(A, np.ones(5))
    assert not st.success() and st.iters() == 0 and st.soln() is None and "p, Ap" in st.msg()
    # the reference reports no residual before breaking down at k = 0 (PCGSolver.py:114-115 returns
    # before :126): empty history, recursive residual = ||b||
    assert len(st.info["hist"]) == 0
    assert st.info["resid_recursive"] == np.sqrt(5.0)


def test_pcg_breakdown_later_history(psk):
    """dot(p, Ap) == 0 at k > 0: the history holds exactly the k residuals reported before it."""
    # A = diag(2, 0, 0), b = (1, 1, 0): step 0 runs (p.Ap = 2) and reports ||r|| = sqrt(2); the next
    # direction lies in the null space, so dot(p, Ap) == 0 at k = 1
    A = sp.csr_matrix(np.array([[2.0, 0.0, 0.0], [0.0, 0.0, 0.0], [0.0, 0.0, 0.0]]))
    b = np.array([1.0, 1.0, 0.0])
    from oracle import krylov
    ref = krylov.pcg(A, b, maxiter=10, tau=1e-8)
    st = psk.PCG(control=_ctl(maxiter=10)).makeSolver().solve(A, b)
    assert st.iters() == ref["iters"] and bool(st.success()) == bool(ref["success"])
    assert len(st.info["hist"]) == len(ref["hist"])
    np.testing.assert_allclose(st.info["hist"], ref["hist"], rtol=1e-14)


@pytest.mark.parametrize("maxiter", [5, 6, 7, 8, 9])
@pytest.mark.parametrize("fail", [True, False])
@pytest.mark.parametrize("jac", ["identity", "jacobi"])
def test_pcg_solution_at_maxiter_odd_even(psk, maxiter, fail, jac):
    """K3 defers x += alpha p (x read and written every kPcgDefer = 4 iterations, p in a ring of 4
    buffers): the solution the loop stops with — at maxiter 5..9, i.e. 0..3 updates pending, with
    and without failOnMaxiter — is the oracle's (to rounding: the device's dot products sum in
    another order than numpy's), and so is the history; a missing or doubled update would be O(1)
    off."""
    from oracle import fdlap, krylov
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, 24)
    b, _ = fdlap.manufactured_rhs(A, 12345)
    pre = psk.Jacobi() if jac == "jacobi" else psk.IdentityPreconditionerType()
    ref = krylov.pcg(A, b, maxiter=maxiter, tau=1e-14, fail_on_maxiter=fail,
                     precond=krylov.jacobi_form(A) if jac == "jacobi" else krylov.identity_apply)
    ctl = psk.CommonSolverArgs(maxiter=maxiter, tau=1e-14, failOnMaxiter=fail, showIters=False, showFinal=False)
    st = psk.PCG(control=ctl, precond=pre).makeSolver().solve(A, b)
    assert st.iters() == ref["iters"] and bool(st.success()) == bool(ref["success"])
    np.testing.assert_allclose(st.soln(), ref["soln"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(st.info["hist"], ref["hist"], rtol=1e-12)


def test_pcg_breakdown_after_even_iteration_flushes_x(psk):
    """A dot(p, Ap) == 0 breakdown at k = 1 leaves iteration 0's deferred x update pending; the C ABI
    still returns x with it applied (x1 = x0 + alpha0 p0, as the reference's loop holds it)."""
    import ctypes
    from pysolvers_amd import _native as N
    A = sp.csr_matrix(np.array([[2.0, 0.0, 0.0], [0.0, 0.0, 0.0], [0.0, 0.0, 0.0]]))
    b = np.array([1.0, 1.0, 0.0])
    dA = psk.DeviceCSR.from_scipy(A)
    ctl = N.PskCtl(maxiter=10, tau=1e-8, fail_on_maxiter=1, restart=0, check_every=0, time_kernels=0)
    res = N.PskResult()
    x = np.full(3, np.nan)
    N.check(N.lib.psk_pcg(dA.handle, None, N.ptr(b), N.ptr(x), ctypes.byref(ctl), ctypes.byref(res), None,
                          N.PSK_HOST), "psk_pcg")
    assert res.status == 2 and res.iters == 1                 # PSK_BREAKDOWN at k = 1
    r0 = b.copy()
    alpha0 = (r0 @ r0) / (r0 @ (A @ r0))                      # p0 = r0, x0 = 0
    assert np.array_equal(x, 0.0 + alpha0 * r0)


def test_torch_tensors_ordered_after_torch_stream(psk):
    """b, x and SpMV/preconditioner operands as torch tensors written by still-queued torch kernels:
    libpsk waits for torch's stream first (same answers as the numpy path)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("torch without a GPU")
    d = load_golden("pcg_fd64_jacobi.npz")
    A = golden_matrix(d)
    dA = psk.DeviceCSR.from_scipy(A)
    s = psk.PCG(control=_ctl(maxiter=4000), precond=psk.Jacobi()).makeSolver()
    st_h = s.solve(dA, d["b"])

    def queued(v):
        # a long chain of torch kernels ahead of the copy that produces the operand
        busy = torch.ones(1 << 24, dtype=torch.float64, device="cuda")
        for _ in range(30):
            busy = busy * 1.0000001
        out = torch.zeros(len(v), dtype=torch.float64, device="cuda")
        out.add_(torch.from_numpy(v).to("cuda", non_blocking=True))
        return out

    st_d = s.solve(dA, queued(d["b"]))
    assert st_d.iters() == st_h.iters()
    assert np.array_equal(st_d.soln().cpu().numpy(), st_h.soln())
    x = np.random.default_rng(5).random(A.shape[0])
    assert np.array_equal(psk.mvmult(dA, queued(x)).cpu().numpy(), A @ x)
    M = psk.Jacobi().form(dA)
    assert np.array_equal(M.applyRight(queued(x)).cpu().numpy(), M.applyRight(x))


def test_pcg_maxiter_zero(psk):
    d = load_golden("pcg_dh8_identity.npz")
    st = psk.PCG(control=_ctl(maxiter=0)).makeSolver().solve(golden_matrix(d), d["b"])
    assert not st.success() and st.iters() == 0


def test_device_resident_vectors(psk):
    """b and x in HBM (DeviceVector): same answer as the host path."""
    d = load_golden("pcg_fd64_jacobi.npz")
    A = psk.DeviceCSR.from_scipy(golden_matrix(d))
    s = psk.PCG(control=_ctl(maxiter=4000), precond=psk.Jacobi()).makeSolver()
    st_h = s.solve(A, d["b"])
    st_d = s.solve(A, psk.DeviceVector.from_numpy(d["b"]))
    assert st_d.iters() == st_h.iters() == 177
    assert np.array_equal(st_d.soln().numpy(), st_h.soln())


def test_frozen_matrix_and_prec_reuse(psk):
    d = load_golden("pcg_dh10_jacobi.npz")
    A = golden_matrix(d)
    s = psk.PCG(control=_ctl(maxiter=2000), precond=psk.Jacobi()).makeSolver()
    s.freezeMatrix()
    s.freezePrec()
    a = s.solve(A, d["b"])
    b = s.solve(A, d["b"])
    assert a.iters() == b.iters() == 103 and np.array_equal(a.soln(), b.soln())


def test_pcg_setup_prints_as_reference(psk, capsys):
    """PCGSolver.solve prints 'prec frozen = ' + precFrozen() on every solve with b != 0 and
    'building prec' whenever it forms the preconditioner (PCGSolver.py:91,93: unconditional prints,
    after the b = 0 early return at :86-88); GMRES prints neither (GMRESSolver.py has no such line)."""
    d = load_golden("pcg_dh8_identity.npz")
    A = golden_matrix(d)
    s = psk.PCG(control=_ctl(maxiter=200)).makeSolver()
    s.solve(A, d["b"])
    assert capsys.readouterr().out == "prec frozen =  False\nbuilding prec\n"
    s.freezePrec()
    s.solve(A, d["b"])
    assert capsys.readouterr().out == "prec frozen =  True\n"
    s.solve(A, np.zeros_like(d["b"]))                        # :86-88 returns before the prints
    assert capsys.readouterr().out == ""
    psk.GMRES(control=_ctl(maxiter=200)).makeSolver().solve(A, d["b"])
    assert capsys.readouterr().out == ""


@pytest.mark.parametrize("case", restarted_cases(), ids=lambda c: c["file"][:-4])
def test_gmres_restarted_matches_reference_cycles(psk, case):
    """GMRES(m) on the device vs the fixtures whose every restart cycle make_restarted.py checked bit
    for bit against the reference's own GMRES solve on the residual system: identical step counts,
    success flags and messages; residual history (one entry per Arnoldi step, across cycles) within
    1e-10 ||b||; solution within 1e-10 relative."""
    d = load_golden(case["file"])
    A = golden_matrix(d)
    ctl = _ctl(maxiter=case["maxiter"], tau=case["tau"], failOnMaxiter=bool(case["fail_on_maxiter"]))
    st = psk.GMRES(control=ctl, precond=product_prec_type(psk, case["precond"]),
                   restart=case["restart"]).makeSolver().solve(A, d["b"])
    assert st.iters() == case["iters"], (st.iters(), case["iters"])
    assert bool(st.success()) == case["success"]
    nb = np.linalg.norm(d["b"])
    h = st.info["hist"]
    assert len(h) == len(d["hist"])
    assert np.max(np.abs(h - d["hist"])) / nb <= RTOL_RESID
    assert abs(st.resid() - case["resid"]) / nb <= RTOL_RESID
    assert np.linalg.norm(st.soln() - d["soln"]) <= 1e-10 * np.linalg.norm(d["soln"])


def test_gmres_maxiter_status(psk):
    d = load_golden("gmres_dh8_identity.npz")
    st = psk.GMRES(control=_ctl(maxiter=10)).makeSolver().solve(golden_matrix(d), d["b"])
    assert not st.success() and st.iters() == 9 and st.msg() == "failure to converge"
    assert np.max(np.abs(st.info["hist"] - d["hist"][:10])) <= RTOL_RESID * np.linalg.norm(d["b"])


# ---------------------------------------------------------------------------------------------
# larger sizes: size-independent properties against the oracle

def test_fd1024_pcg_jacobi_iterations(psk):
    d = load_golden("large_fd1024.npz")
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, 1024)
    b = psk.mvmult(dA, np.random.default_rng(12345).random(1024 * 1024))
    assert np.array_equal(b[:4096], d["b_head"])
    assert hashlib.sha256(b.tobytes()).hexdigest() == str(d["b_sha256"])
    st = psk.PCG(control=_ctl(maxiter=4000), precond=psk.Jacobi()).makeSolver().solve(dA, b)
    assert st.iters() == int(d["iters"])
    nb = np.linalg.norm(b)
    th = max(RTOL_RESID, 10 * float(d["sens_hist"]))
    assert np.max(np.abs(st.info["hist"] - d["hist"])) / nb <= th
    assert abs(st.resid() - float(d["resid"])) / nb <= th
    tx = max(1e-10, 10 * float(d["sens_x"]))
    x = st.soln()
    assert np.linalg.norm(x[:4096] - d["soln_head"]) <= tx * float(d["soln_norm"])


def test_fd4096_pcg_jacobi_iterations(psk):
    """configs[1] (PCG + Jacobi, FD 4096^2) to convergence at tau = 1e-8: the iteration count the
    reference path takes (5813, tests/golden/make_large_oracle.py: the oracle, bit-identical to the
    reference on every fixture; its 1-ulp dot perturbations keep 5813 and move the history by
    8.6e-17 ||b||) must be identical; history within 1e-10 ||b||; solution within 1e-10."""
    d = load_golden("large_fd4096.npz")
    m = int(d["m"])
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    b = psk.mvmult(dA, np.random.default_rng(12345).random(m * m))
    assert np.array_equal(b[:4096], d["b_head"])
    assert hashlib.sha256(b.tobytes()).hexdigest() == str(d["b_sha256"])
    st = psk.PCG(control=_ctl(maxiter=40000), precond=psk.Jacobi()).makeSolver().solve(dA, b)
    assert st.success() and st.iters() == int(d["iters"]) == 5813
    nb = np.linalg.norm(b)
    th = max(RTOL_RESID, 10 * float(d["sens_hist"]))
    assert np.max(np.abs(st.info["hist"] - d["hist"])) / nb <= th
    assert abs(st.resid() - float(d["resid"])) / nb <= th
    tx = max(1e-10, 10 * float(d["sens_x"]))
    assert np.linalg.norm(st.soln()[:4096] - d["soln_head"]) <= tx * float(d["soln_norm"])


def test_fd4096_spmv_and_first_iterations(psk):
    """configs[1] size (n = 16.7M): SpMV bit-exact vs the C oracle, 12 PCG+Jacobi steps vs the numpy oracle."""
    from oracle import fdlap, krylov, native
    m = 4096
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    x = np.random.default_rng(12345).random(m * m)
    b = psk.mvmult(dA, x)
    assert np.array_equal(b, native.csr_matvec(A, x))
    ctl = _ctl(maxiter=12, tau=0.0, failOnMaxiter=False)
    st = psk.PCG(control=ctl, precond=psk.Jacobi()).makeSolver().solve(dA, b)
    ref = krylov.pcg(A, b, maxiter=12, tau=0.0, fail_on_maxiter=False, precond=krylov.jacobi_form(A))
    assert st.iters() == ref["iters"] == 12
    np.testing.assert_allclose(st.info["hist"], ref["hist"], rtol=RTOL_RESID)
    assert np.linalg.norm(st.soln() - ref["soln"]) <= 1e-12 * np.linalg.norm(ref["soln"])


# m chosen so the one-shot grids straddle the gridsum geometry (psk_internal.hpp): SpMV tiles
# ceil(m^2/256) = 255 / 256 (one level) / 259 (groups) / 4727 (groups with lagged AND own-group
# reducers); K2/K3 tiles ceil(m^2/512) likewise
@pytest.mark.parametrize("m", [255, 256, 257, 363, 1100])
def test_pcg_gridsum_geometries(psk, m):
    from oracle import fdlap, krylov
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    dA = psk.DeviceCSR.from_scipy(A)
    b = A @ np.random.default_rng(m).random(m * m)
    ctl = _ctl(maxiter=12, tau=0.0, failOnMaxiter=False)
    for prec, oprec in ((psk.Jacobi(), krylov.jacobi_form(A)), (None, krylov.identity_apply)):
        kw = {"precond": prec} if prec is not None else {}
        st = psk.PCG(control=ctl, **kw).makeSolver().solve(dA, b)
        ref = krylov.pcg(A, b, maxiter=12, tau=0.0, fail_on_maxiter=False, precond=oprec)
        assert st.iters() == ref["iters"] == 12
        np.testing.assert_allclose(st.info["hist"], ref["hist"], rtol=RTOL_RESID)
        assert np.linalg.norm(st.soln() - ref["soln"]) <= 1e-12 * np.linalg.norm(ref["soln"])


def test_pcg_run_to_run_bitwise(psk):
    """The in-launch reductions have a fixed order: two solves of the same system agree bit for bit."""
    m = 1100
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    b = psk.mvmult(dA, np.random.default_rng(7).random(m * m))
    ctl = _ctl(maxiter=50, tau=0.0, failOnMaxiter=False)
    s1 = psk.PCG(control=ctl, precond=psk.Jacobi()).makeSolver().solve(dA, b)
    s2 = psk.PCG(control=ctl, precond=psk.Jacobi()).makeSolver().solve(dA, b)
    assert np.array_equal(s1.soln(), s2.soln())
    assert np.array_equal(s1.info["hist"], s2.info["hist"])


# ---------------------------------------------------------------------------------------------
# ILUT apply (RightILUTPreconditioner.applyRight = SuperLU ILU.solve) on the device

@pytest.mark.parametrize("tag", ["fd64", "dh8"])
def test_ilut_apply_matches_superlu(psk, tag):
    d = load_golden("spmv.npz")
    A = golden_matrix(d, tag + "_")
    M = psk.RightILUT().form(A)
    v = d[tag + "_x"]
    ref = M.ILU().solve(v)
    out = M.applyRight(v)
    assert np.linalg.norm(out - ref) <= 1e-13 * np.linalg.norm(ref)
    assert np.array_equal(M.applyLeft(v), v)                  # right preconditioner: identity on the left
    L = psk.LeftILUT().form(A)
    assert np.array_equal(L.applyRight(v), v)                 # Preconditioner.py:44-45
    assert np.linalg.norm(L.applyLeft(v) - ref) <= 1e-13 * np.linalg.norm(ref)


def test_ilut_apply_large_fd():
    """FD m=512 (262k rows, ~3.7k dependency levels): device sweep vs SuperLU ILU.solve."""
    import pysolvers_amd as psk
    from oracle import fdlap
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, 512)
    M = psk.RightILUT().form(A)
    v = np.random.default_rng(9).standard_normal(A.shape[0])
    ref = M.ILU().solve(v)
    assert np.linalg.norm(M.applyRight(v) - ref) <= 1e-12 * np.linalg.norm(ref)


# ---------------------------------------------------------------------------------------------
# CommonSolverArgs.norm other than numpy.linalg.norm (IterativeSolver.py:86-88)

def _inf_norm(v):
    return np.linalg.norm(v, np.inf)


def _one_norm(v):
    return np.abs(v).sum()


@pytest.mark.parametrize("case,norm", [("pcg_dh10_identity.npz", _inf_norm), ("pcg_fd32_identity.npz", _one_norm),
                                       ("pcg_fd64_jacobi.npz", _inf_norm)])
def test_pcg_caller_norm_matches_oracle(psk, case, norm):
    """A caller-supplied norm (PCGSolver.py:86 ||b||, :125 ||r|| every iteration): the host-driven loop
    over the device kernels takes the oracle's iteration count; residual history within 1e-10 of the
    norm of b, solution within 1e-10."""
    from oracle import krylov
    d = load_golden(case)
    A = golden_matrix(d)
    prec = "jacobi" if "jacobi" in case else "identity"
    ctl = _ctl(maxiter=4000, tau=1e-8, norm=norm)
    st = psk.PCG(control=ctl, precond=product_prec_type(psk, prec)).makeSolver().solve(A, d["b"])
    ref = krylov.pcg(A, d["b"], maxiter=4000, tau=1e-8, precond=oracle_prec(A, prec), norm=norm)
    assert st.iters() == ref["iters"] and bool(st.success()) == bool(ref["success"])
    nb = norm(d["b"])
    assert len(st.info["hist"]) == len(ref["hist"])
    assert np.max(np.abs(st.info["hist"] - ref["hist"])) <= 1e-10 * nb
    assert np.linalg.norm(st.soln() - ref["soln"]) <= 1e-10 * np.linalg.norm(ref["soln"])


@pytest.mark.parametrize("case", ["gmres_dh8_identity.npz", "gmres_fd16_jacobi.npz"])
def test_gmres_caller_norm_matches_oracle(psk, case):
    """GMRES with a caller-supplied norm: threshold tau * norm(b) (GMRESSolver.py:66) and the true
    residual test norm(b - A x) (:164) in that norm; the Arnoldi norms stay npla.norm (:90, :115, :121)."""
    from oracle import krylov
    d = load_golden(case)
    A = golden_matrix(d)
    prec = "jacobi" if "jacobi" in case else "identity"
    for norm, tau in ((_inf_norm, 1e-8), (_one_norm, 1e-9)):
        ctl = _ctl(maxiter=300, tau=tau, norm=norm)
        st = psk.GMRES(control=ctl, precond=product_prec_type(psk, prec)).makeSolver().solve(A, d["b"])
        ref = krylov.gmres(A, d["b"], maxiter=300, tau=tau, precond=oracle_prec(A, prec), norm=norm)
        assert st.iters() == ref["iters"] and bool(st.success()) == bool(ref["success"])
        assert np.max(np.abs(st.info["hist"] - ref["hist"])) <= 1e-10 * np.linalg.norm(d["b"])
        assert abs(st.resid() - ref["resid"]) <= 1e-10 * norm(d["b"])
        assert np.linalg.norm(st.soln() - ref["soln"]) <= 1e-10 * np.linalg.norm(ref["soln"])


def test_caller_norm_zero_rhs(psk):
    d = load_golden("pcg_dh8_identity.npz")
    A = golden_matrix(d)
    for f in (psk.PCG, psk.GMRES):
        st = f(control=_ctl(maxiter=50, norm=_inf_norm)).makeSolver().solve(A, np.zeros(A.shape[0]))
        assert st.success() and st.iters() == 1 and not np.any(st.soln())


def test_caller_norm_keeps_the_vector_kind(psk):
    """A CUDA-tensor right-hand side gets a CUDA tensor back on every path — the device loop, the
    host-driven caller-norm PCG and its b = 0 early return — and the same numbers."""
    import torch
    d = load_golden("pcg_dh8_identity.npz")
    A = golden_matrix(d)
    bt = torch.as_tensor(d["b"], dtype=torch.float64, device="cuda")
    for ctl in (_ctl(maxiter=4000, tau=1e-8), _ctl(maxiter=4000, tau=1e-8, norm=_inf_norm)):
        st = psk.PCG(control=ctl).makeSolver().solve(A, bt)
        sh = psk.PCG(control=ctl).makeSolver().solve(A, d["b"])
        assert torch.is_tensor(st.soln()) and st.soln().is_cuda and isinstance(sh.soln(), np.ndarray)
        assert np.array_equal(st.soln().cpu().numpy(), sh.soln()) and st.iters() == sh.iters()
    z = psk.PCG(control=_ctl(maxiter=50, norm=_inf_norm)).makeSolver().solve(A, torch.zeros_like(bt))
    assert torch.is_tensor(z.soln()) and z.soln().is_cuda and not bool(torch.any(z.soln() != 0))


def test_gmres_exit_reason(psk):
    """psk_result.exit (ABI 3) says why the loop stopped; the caller-norm true-residual re-test is
    gated on it, not on the history length."""
    import ctypes
    from pysolvers_amd import _native as N
    d = load_golden("gmres_dh8_identity.npz")
    dA = psk.DeviceCSR.from_scipy(golden_matrix(d))
    b = np.ascontiguousarray(d["b"])
    for maxiter, fom, want in ((300, 1, N.PSK_EXIT_TOLERANCE), (10, 1, N.PSK_EXIT_MAXITER),
                               (10, 0, N.PSK_EXIT_MAXITER)):
        ctl = N.PskCtl(maxiter=maxiter, tau=1e-8, fail_on_maxiter=fom, restart=0, check_every=0, time_kernels=0)
        res, x = N.PskResult(), np.empty_like(b)
        N.check(N.lib.psk_gmres(dA.handle, None, N.ptr(b), N.ptr(x), ctypes.byref(ctl), ctypes.byref(res), None,
                                N.PSK_HOST), "psk_gmres")
        assert res.exit == want, (maxiter, fom, res.exit)
    res, x, z = N.PskResult(), np.empty_like(b), np.zeros_like(b)
    ctl = N.PskCtl(maxiter=10, tau=1e-8, fail_on_maxiter=1, restart=0, check_every=0, time_kernels=0)
    N.check(N.lib.psk_gmres(dA.handle, None, N.ptr(z), N.ptr(x), ctypes.byref(ctl), ctypes.byref(res), None,
                            N.PSK_HOST), "psk_gmres")
    assert res.exit == N.PSK_EXIT_NONE and res.success == 1
