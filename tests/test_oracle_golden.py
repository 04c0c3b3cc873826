"""The oracle (CPU restatement) against the golden vectors produced by the reference itself.

tests/golden/make_golden.py ran the reference (krlong014/PySolvers) and asserted
bit-identity with the oracle in the build container; these tests re-check the
oracle against the committed vectors wherever the suite runs (another host's
OpenBLAS may order its dot products differently, so solver outputs are compared
with tight tolerances while SpMV / generator / Givens outputs must be exact).
"""
import hashlib

import numpy as np
import pytest

from conftest import (case_precond, dense_cases, golden_matrix, load_golden, manifest, oracle_prec, product_prec_type,
                      restarted_cases, solver_cases)
from oracle import fdlap, krylov, native


def _sha(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("m", [1, 2, 3, 5, 16])
def test_fd_generator_arrays_exact(m):
    d = load_golden("fd_generator.npz")
    ip, ix, dt = fdlap.fd_laplacian_2d_arrays(-1.0, 1.0, m)
    assert np.array_equal(ip, d["m%d_indptr" % m])
    assert np.array_equal(ix, d["m%d_indices" % m])
    assert np.array_equal(dt, d["m%d_data" % m])
    assert np.array_equal(fdlap.fd_rowptr_closed_form(m, np.arange(m * m + 1)), ip)


@pytest.mark.parametrize("m", ["64", "128", "300"])
def test_fd_generator_hash(m):
    ref = manifest()["fd_generator_sha256"][m]
    ip, ix, dt = fdlap.fd_laplacian_2d_arrays(-1.0, 1.0, int(m))
    assert len(dt) == ref["nnz"]
    assert _sha(ip, ix, dt) == ref["sha256"]


@pytest.mark.parametrize("tag", ["fd64", "dh8"])
def test_spmv_exact(tag):
    d = load_golden("spmv.npz")
    A = golden_matrix(d, tag + "_")
    y_ref = d[tag + "_y"]
    assert np.array_equal(A @ d[tag + "_x"], y_ref)                       # scipy csr_matvec
    assert np.array_equal(native.csr_matvec(A, d[tag + "_x"]), y_ref)     # plain-C restatement


@pytest.mark.parametrize("m", [1, 2, 3, 5, 64, 300])
def test_fd_stencil_matches_csr_matvec(m):
    """oracle.fdlap.FDStencil (the matrix-free restatement the 16384^2 GPU tests use) against scipy
    csr_matvec on the reference generator's CSR: bit for bit, including signed zeros."""
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    S = fdlap.FDStencil(-1.0, 1.0, m)
    assert S.shape == A.shape
    assert np.array_equal(S.diagonal(), A.diagonal())
    rng = np.random.default_rng(m)
    for x in (rng.random(m * m), rng.standard_normal(m * m), np.where(rng.random(m * m) < 0.5, -0.0, 0.0)):
        y, yr = S @ x, A @ x
        assert np.array_equal(y.view(np.int64), yr.view(np.int64))
    if m == 64:
        d = load_golden("spmv.npz")
        assert np.array_equal(S @ d["fd64_x"], d["fd64_y"])


def test_csr_diagonal_exact():
    d = load_golden("spmv.npz")
    for tag in ("fd64", "dh8"):
        A = golden_matrix(d, tag + "_")
        assert np.array_equal(native.csr_diagonal(A), A.diagonal())


def test_givens_selftest_exact():
    d = load_golden("givens.npz")
    H, g, CS, y = krylov.givens_triangularize(d["H"], d["g"])
    assert np.array_equal(H, d["H_rot"]) and np.array_equal(g, d["g_rot"])
    assert np.array_equal(CS, d["CS"]) and np.array_equal(y, d["y"])


@pytest.mark.parametrize("case", solver_cases(), ids=lambda c: c["file"][:-4])
def test_oracle_solvers_match_reference(case):
    d = load_golden(case["file"])
    A = golden_matrix(d)
    b = d["b"]
    assert np.array_equal(A @ d["x_exact"], b)
    prec = oracle_prec(A, case_precond(case))
    fn = krylov.pcg if case["kind"] == "pcg" else krylov.gmres
    st = fn(A, b, maxiter=case["maxiter"], tau=case["tau"], fail_on_maxiter=bool(case["fail_on_maxiter"]),
            precond=prec)
    assert st["iters"] == case["iters"]
    assert bool(st["success"]) == case["success"]
    h = d["hist"]
    assert len(st["hist"]) == len(h)
    np.testing.assert_allclose(st["hist"], h, rtol=1e-10, atol=0)
    if d["soln"].size:
        np.testing.assert_allclose(st["soln"], d["soln"], rtol=1e-9, atol=1e-12 * np.abs(d["soln"]).max())


@pytest.mark.parametrize("case", restarted_cases(), ids=lambda c: c["file"][:-4])
def test_oracle_restarted_gmres_matches_fixture(case):
    """GMRES(m) restatement (cycles of GMRESSolver.py:87-160 on the residual system) against the
    fixtures make_restarted.py pinned cycle by cycle to the reference's own solve."""
    d = load_golden(case["file"])
    A = golden_matrix(d)
    b = d["b"]
    prec = oracle_prec(A, case["precond"])
    st = krylov.gmres_restarted(A, b, case["restart"], maxiter=case["maxiter"], tau=case["tau"],
                                fail_on_maxiter=bool(case["fail_on_maxiter"]), precond=prec)
    assert st["iters"] == case["iters"] and bool(st["success"]) == case["success"]
    assert len(st["hist"]) == len(d["hist"])
    np.testing.assert_allclose(st["hist"], d["hist"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(st["soln"], d["soln"], rtol=1e-9, atol=1e-12 * np.abs(d["soln"]).max())


def test_restarted_equals_reference_when_one_cycle_suffices():
    """restart >= the steps needed: GMRES(m) IS the reference's non-restarted solve (same golden)."""
    d = load_golden("gmres_dh8_identity.npz")
    A = golden_matrix(d)
    st = krylov.gmres_restarted(A, d["b"], 300, maxiter=300, tau=1e-8)
    assert st["iters"] == int(d["iters"])
    assert np.array_equal(st["hist"], d["hist"]) and np.array_equal(st["soln"], d["soln"])


def test_zero_rhs_convention():
    d = load_golden("pcg_dh8_identity.npz")
    A = golden_matrix(d)
    for fn in (krylov.pcg, krylov.gmres):
        st = fn(A, np.zeros(A.shape[0]))
        assert st["iters"] == manifest()["zero_rhs"]["iters"] and st["success"]
        assert not np.any(st["soln"])


@pytest.mark.parametrize("case", manifest().get("newton", []), ids=lambda c: c["file"][:-4])
def test_oracle_newton_matches_reference(case):
    """NewtonSolver + PCG on FD-Bratu (examples/FDBratu2D.py): the oracle restatement reproduces the
    reference's Newton residual history, per-step PCG iteration counts and solution bit for bit."""
    from oracle import amg, newton
    d = load_golden(case["file"])
    m = case["m"]
    fp = (lambda J: krylov.ic_form(J)) if case["precond"] == "ic" else (lambda J: amg.AMGApply(J, num_iters=5))
    st = newton.newton(newton.Bratu2D(m=m), np.ones(m * m), fp, maxiter=10, tau=1e-12, min_lin_tol=1e-6)
    assert st["iters"] == case["iters"] and bool(st["success"]) == case["success"]
    assert st["linear_iters"] == case["linear_iters"]
    assert np.array_equal(st["hist"], d["hist"])
    if d["soln"].size:
        assert np.array_equal(st["soln"], d["soln"])


def test_oracle_newton_default_direct_matches_reference():
    """NewtonSolver with its default linear solver (DefaultDirect: spsolve, Newton.py:13): the oracle
    reproduces the reference's history, count and solution bit for bit (make_direct.py)."""
    from conftest import direct_manifest
    from oracle import newton
    for case in direct_manifest()["newton_direct"]:
        d = load_golden(case["file"])
        m = case["m"]
        st = newton.newton(newton.Bratu2D(m=m), np.ones(m * m), None, maxiter=10, tau=1e-12, direct=True)
        assert st["iters"] == case["iters"] and bool(st["success"]) == case["success"]
        np.testing.assert_allclose(st["hist"], d["hist"], rtol=1e-12, atol=0)
        np.testing.assert_allclose(st["soln"], d["soln"], rtol=1e-12, atol=0)


def test_direct_singular_fixture_is_spsolve():
    """The singular-input fixtures make_direct.py took from the reference's DefaultDirect are what
    scipy's spsolve (the reference's call, DefaultDirectSolver.py:65) does: warn, return NaNs."""
    import warnings
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    from conftest import direct_manifest
    for case in direct_manifest()["singular"]:
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            x = spla.spsolve(sp.csr_matrix(np.array(case["dense"])), np.array(case["b"]))
        assert case["success"] and bool(np.all(np.isnan(x))) == case["soln_all_nan"]
        assert sorted({type(i.message).__name__ for i in w}) == case["warnings"]


@pytest.mark.parametrize("case", dense_cases(), ids=lambda c: c["file"][:-4])
def test_oracle_dense_solvers_match_reference(case):
    """A dense ndarray A (IterativeLinearSolver.py:105-106, np.dot): the oracle's A @ x path against the
    reference's run (make_dense.py asserted bit-identity in the build container; here to 1e-10)."""
    d = load_golden(case["file"])
    A, b = d["A"], d["b"]
    assert isinstance(A, np.ndarray) and A.ndim == 2
    assert np.allclose(A @ d["x_exact"], b, rtol=1e-14, atol=1e-14 * np.abs(b).max())
    prec = oracle_prec(A, case_precond(case))
    fn = krylov.pcg if case["kind"] == "pcg" else krylov.gmres
    st = fn(A, b, maxiter=case["maxiter"], tau=case["tau"], fail_on_maxiter=bool(case["fail_on_maxiter"]),
            precond=prec)
    assert st["iters"] == case["iters"] and bool(st["success"]) == case["success"]
    assert len(st["hist"]) == len(d["hist"])
    np.testing.assert_allclose(st["hist"], d["hist"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(st["soln"], d["soln"], rtol=1e-9, atol=1e-12 * np.abs(d["soln"]).max())
