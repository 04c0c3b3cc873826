"""AMG setup on the host (no GPU): SmoothedAggregation.py restated in O(nnz), bit-identical.

* oracle/amg.py against the reference's own hierarchy and apply outputs (tests/golden/amg_hierarchy.npz,
  written by make_golden.py, which asserted reference == oracle bitwise when it ran);
* the product setup (pysolvers_amd.Linear.SmoothedAggregation, psk_sa_aggregate in C++) against
  the same fixtures and against the oracle on matrices the fixtures do not cover (isolated nodes,
  weak couplings, mixed signs, unsorted rows);
* the coarse-level solve factorisation: SuperLU of A_c^T solved transposed == spsolve(A_c, f).
"""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from conftest import load_golden, manifest
from oracle import amg

KEYS = [d["key"] for d in manifest()["amg_hierarchy"]]


def _fix_matrix(d, key, tag):
    shape = tuple(int(s) for s in d["%s_%s_shape" % (key, tag)])
    return sp.csr_matrix((d["%s_%s_data" % (key, tag)], d["%s_%s_indices" % (key, tag)],
                          d["%s_%s_indptr" % (key, tag)]), shape=shape)


def _bitwise(A, B):
    A, B = sp.csr_matrix(A), sp.csr_matrix(B)
    return (A.shape == B.shape and np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
            and np.array_equal(A.data.view(np.uint64), B.data.view(np.uint64)))


@pytest.fixture(scope="module")
def fix():
    return load_golden("amg_hierarchy.npz")


@pytest.mark.parametrize("key", KEYS)
def test_oracle_hierarchy_matches_reference(fix, key):
    L = int(key.split("_L")[1])
    A = _fix_matrix(fix, key, "A%d" % (L - 1))
    ops, P, R = amg.hierarchy(A, L)
    for k in range(L):
        assert _bitwise(ops[k], _fix_matrix(fix, key, "A%d" % k)), k
    for k in range(L - 1):
        assert _bitwise(P[k], _fix_matrix(fix, key, "P%d" % k)), k
        assert _bitwise(R[k], _fix_matrix(fix, key, "R%d" % k)), k
    for sm in ("gs", "jacobi"):
        y = amg.AMGApply(A, num_iters=2, num_levels=L, smoother=sm)(fix[key + "_v"])
        assert np.array_equal(y, fix["%s_apply_%s" % (key, sm)]), sm


@pytest.mark.parametrize("key", KEYS)
def test_product_hierarchy_matches_reference(fix, key):
    from pysolvers_amd.Linear import SmoothedAggregationMLHierarchy
    L = int(key.split("_L")[1])
    A = _fix_matrix(fix, key, "A%d" % (L - 1))
    h = SmoothedAggregationMLHierarchy(A, numLevels=L)
    for k in range(L):
        assert _bitwise(h.matrix(k), _fix_matrix(fix, key, "A%d" % k)), k
    for k in range(L - 1):
        assert _bitwise(h.update(k), _fix_matrix(fix, key, "P%d" % k)), k
        assert _bitwise(h.downdate(k), _fix_matrix(fix, key, "R%d" % k)), k


def _random_matrix(n, seed, density=0.02, isolated=0, weak_scale=1e-3, shuffle=True):
    """Symmetric sparse matrix with strong and weak couplings, some isolated rows, unsorted rows."""
    rng = np.random.default_rng(seed)
    M = sp.random(n, n, density=density, random_state=rng, format="coo")
    vals = -np.abs(M.data) * np.where(rng.random(M.data.shape[0]) < 0.3, weak_scale, 1.0)
    vals *= np.where(rng.random(M.data.shape[0]) < 0.1, -1.0, 1.0)          # a few positive couplings
    M = sp.coo_matrix((vals, (M.row, M.col)), shape=(n, n))
    M = (M + M.T).tocsr()
    M.setdiag(0)
    M.eliminate_zeros()
    iso = rng.choice(n, size=isolated, replace=False) if isolated else np.array([], dtype=int)
    keep = ~(np.isin(M.tocoo().row, iso) | np.isin(M.tocoo().col, iso))
    C = M.tocoo()
    M = sp.coo_matrix((C.data[keep], (C.row[keep], C.col[keep])), shape=(n, n)).tocsr()
    d = np.asarray(np.abs(M).sum(axis=1)).ravel() + 1.0
    A = (M + sp.diags(d)).tocsr()
    if shuffle:                       # unsorted stored order inside rows (like the FD generator)
        A = A.copy()
        for i in range(n):
            s, e = A.indptr[i], A.indptr[i + 1]
            p = s + rng.permutation(e - s)
            A.indices[s:e], A.data[s:e] = A.indices[p].copy(), A.data[p].copy()
        A.has_sorted_indices = False
    return A


CASES = [("rand300", _random_matrix(300, 1)), ("rand500_iso", _random_matrix(500, 2, isolated=7)),
         ("rand400_dense", _random_matrix(400, 3, density=0.05, weak_scale=0.05)),
         ("rand200_sorted", _random_matrix(200, 4, shuffle=False))]


@pytest.mark.parametrize("name,A", CASES, ids=[c[0] for c in CASES])
def test_native_aggregation_matches_oracle(name, A):
    from pysolvers_amd.Linear.SmoothedAggregation import BuildAggregates
    for lvl in (1, 2):
        tol = amg.default_tol(lvl)
        agg, count, afv = BuildAggregates(A, lvl=lvl)
        oagg, ocount, root, late = amg.build_aggregates(A, tol)
        assert count == ocount
        assert np.array_equal(agg, oagg)
        Af = amg.filtered_matrix(A, amg.filter_mask(A, amg.strong_mask(A, tol), oagg, root, late))
        assert np.array_equal(afv.view(np.uint64), Af.data.view(np.uint64))


@pytest.mark.parametrize("name,A", CASES, ids=[c[0] for c in CASES])
def test_native_hierarchy_matches_oracle(name, A):
    from pysolvers_amd.Linear import SmoothedAggregationMLHierarchy
    for L in (2, 3):
        h = SmoothedAggregationMLHierarchy(A, numLevels=L)
        ops, P, R = amg.hierarchy(A, L)
        for k in range(L):
            assert _bitwise(h.matrix(k), ops[k])
        for k in range(L - 1):
            assert _bitwise(h.update(k), P[k]) and _bitwise(h.downdate(k), R[k])


def test_restriction_is_transpose_without_normalisation(fix):
    from pysolvers_amd.Linear import makeRestrictionOp
    P = _fix_matrix(fix, "dh8_L2", "P0")
    R = makeRestrictionOp(P)
    assert _bitwise(R, _fix_matrix(fix, "dh8_L2", "R0"))
    T = P.T.tocsr()
    T.sort_indices()
    assert _bitwise(R, T)


@pytest.mark.parametrize("key", ["dh10_L2", "negfd32_L2", "dh8_L3"])
def test_coarse_factorisation_is_spsolve(fix, key):
    """VCycleManager.py:36 spsolve(A_c, f) == splu(A_c^T).solve(f, 'T') bitwise, and the device
    chain's restatement (gather perm_c^-1, U^T lower, L^T unit upper, gather perm_r) agrees."""
    from pysolvers_amd.Linear.AMGPreconditioner import coarse_factor
    from pysolvers_amd.Linear.TriangularSolve import inverse_permutation
    A0 = _fix_matrix(fix, key, "A0")
    lu = coarse_factor(A0)
    f = np.random.default_rng(5).standard_normal(A0.shape[0])
    x_ref = spla.spsolve(A0.copy(), f)
    assert np.array_equal(lu.solve(f, trans="T"), x_ref)
    n = A0.shape[0]
    Ut = sp.csr_matrix((lu.U.data, lu.U.indices, lu.U.indptr), shape=(n, n))
    Lt = sp.csr_matrix((lu.L.data, lu.L.indices, lu.L.indptr), shape=(n, n))
    y = spla.spsolve_triangular(Ut, f[inverse_permutation(lu.perm_c)], lower=True)
    z = spla.spsolve_triangular(Lt, y, lower=False, unit_diagonal=True)
    np.testing.assert_allclose(z[lu.perm_r], x_ref, rtol=0, atol=1e-12 * np.abs(x_ref).max())


def test_native_first_level_matches_oracle_negfd1024():
    """configs[4]'s matrix family at 1M rows (-FDLaplacian2D 1024^2, FDBratu2D.py:15 sign): the native
    O(nnz) aggregation, the filtered matrix and the smoothed prolongator of the first coarsening
    equal the oracle's restatement bit for bit (the GPU suite runs the 8192^2 hierarchy itself)."""
    from oracle import fdlap
    from pysolvers_amd.Linear.SmoothedAggregation import SA_coarsen
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, 1024)
    P, agg = SA_coarsen(A, lvl=1)
    oP, oagg = amg.sa_coarsen(A, lvl=1)
    assert np.array_equal(agg, oagg)
    assert _bitwise(P, oP)


def test_amg_coarse_option_validated_before_any_device_work():
    """AMG(coarse=...) accepts "auto" / "dense" / "lu" (the dense coarse solve, round 5); anything else is
    refused before a device matrix is created, so this runs without a GPU."""
    import pysolvers_amd as psk
    A = sp.identity(4, format="csr")
    with pytest.raises(ValueError):
        psk.AMG(coarse="qr").form(A)


def test_dense_coarse_accuracy_model_on_host():
    """What the dense coarse solve relies on, checked on the host for an SA coarse operator of -FD 256^2
    (n_c ~ 1,000): x = A_c^-1 f through an explicit inverse agrees with SuperLU's transposed solve (the
    reference's spsolve) far inside the 1e-12 the GPU tests pin."""
    from oracle import fdlap
    from pysolvers_amd.Linear.AMGPreconditioner import coarse_factor
    from pysolvers_amd.Linear.SmoothedAggregation import SmoothedAggregationMLHierarchy
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, 256)
    Ac = sp.csr_matrix(SmoothedAggregationMLHierarchy(sp.csr_matrix(A), numLevels=3).matrix(0))
    lu = coarse_factor(Ac)
    Minv = np.linalg.inv(Ac.toarray())
    f = np.random.default_rng(0).standard_normal(Ac.shape[0])
    xs = lu.solve(f, trans='T')
    assert np.max(np.abs(Minv @ f - xs)) <= 1e-13 * np.max(np.abs(xs))
