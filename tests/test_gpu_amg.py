"""GPU parity of the triangular-solve chains (IC, Gauss-Seidel, coarse LU) and the AMG V-cycle.

Bars (written here, not inferred):
* AMG apply vs the reference's own outputs (amg_hierarchy.npz): ||y - y_ref|| <= 1e-10 ||y_ref||.
  Not bitwise: the triangular solves sum each row with FMA in stored order where SuperLU uses its
  supernodal column order; SpMV, restriction, prolongation and Jacobi sweeps are bitwise.
* RightIC apply vs the reference's spsolve_triangular pair: 1e-12 relative.
* generic chains vs scipy on random factors with permutations: 1e-12 relative.
Solver-level parity of PCG/GMRES + AMG / RightIC runs in test_gpu_parity.test_solver_matches_reference
(the golden manifest carries those cases).
"""
import functools

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from conftest import load_golden, manifest

pytestmark = pytest.mark.gpu

KEYS = [d["key"] for d in manifest()["amg_hierarchy"]]


@pytest.fixture(scope="module")
def psk():
    import pysolvers_amd
    return pysolvers_amd


@pytest.fixture(scope="module")
def fix():
    return load_golden("amg_hierarchy.npz")


def _fix_matrix(d, key, tag):
    shape = tuple(int(s) for s in d["%s_%s_shape" % (key, tag)])
    return sp.csr_matrix((d["%s_%s_data" % (key, tag)], d["%s_%s_indices" % (key, tag)],
                          d["%s_%s_indptr" % (key, tag)]), shape=shape)


def _rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.mark.parametrize("key", KEYS)
@pytest.mark.parametrize("sm", ["gs", "jacobi"])
def test_amg_apply_matches_reference(psk, fix, key, sm):
    L = int(key.split("_L")[1])
    A = _fix_matrix(fix, key, "A%d" % (L - 1))
    kw = {"smoother": psk.JacobiSmoother} if sm == "jacobi" else {}
    M = psk.AMG(numIters=2, numLevels=L, **kw).form(A)
    assert M.levels() == [int(_fix_matrix(fix, key, "A%d" % k).shape[0]) for k in range(L)]
    y_ref = fix["%s_apply_%s" % (key, sm)]
    v = fix[key + "_v"]
    y = M.applyRight(v)
    assert _rel(y, y_ref) <= 1e-10, _rel(y, y_ref)
    assert np.array_equal(M.applyLeft(v), y)                 # GenericPreconditioner: same both sides
    yd = M.apply(psk.DeviceVector.from_numpy(v)).numpy()     # device-resident vectors
    assert np.array_equal(yd, y)


def test_amg_early_exit_matches_oracle(psk):
    """numIters large enough that the 1e-8 test stops the cycles early (VCycleSolver.py:141-142)."""
    from oracle import amg
    d = load_golden("pcg_dh8_amg.npz")
    from conftest import golden_matrix
    A = golden_matrix(d)
    v = np.random.default_rng(3).standard_normal(A.shape[0])
    ref = amg.AMGApply(A, num_iters=40, num_levels=2)
    # how many cycles the oracle runs before the test holds
    x = v.copy()
    ncyc = None
    for k in range(40):
        x = amg.vcycle(ref.ops, ref.P, ref.R, ref.aux, "gs", v, x, 1)
        if np.linalg.norm(v - A @ x) < 1e-8 * np.linalg.norm(v):
            ncyc = k + 1
            break
    assert ncyc is not None and ncyc < 40
    y = psk.AMG(numIters=40).form(A).applyRight(v)
    assert _rel(y, ref(v)) <= 1e-10
    assert _rel(y, x) <= 1e-10          # the snapshot after cycle ncyc, not the 40-cycle iterate


def test_amg_zero_rhs(psk, fix):
    A = _fix_matrix(fix, "dh8_L2", "A1")
    M = psk.AMG(numIters=2).form(A)
    y = M.applyRight(np.zeros(A.shape[0]))
    assert not np.any(y)


@pytest.mark.parametrize("m", [128, 384])
def test_amg_apply_negfd_vs_oracle(psk, m):
    """-FD2D (FDBratu2D.py:15), 2 and 3 levels, against the oracle (pinned bitwise to the reference
    on the fixtures; the reference's own setup is quadratic, 253 s at m=512)."""
    from oracle import amg, fdlap
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    v = np.random.default_rng(11).standard_normal(A.shape[0])
    for L in (2, 3):
        M = psk.AMG(numIters=2, numLevels=L).form(A)
        ref = amg.AMGApply(A, num_iters=2, num_levels=L)
        assert M.levels() == [o.shape[0] for o in ref.ops]
        assert _rel(M.applyRight(v), ref(v)) <= 1e-10


@pytest.mark.parametrize("case", ["pcg_dh10_ic.npz", "pcg_negfd32_ic.npz"])
def test_ic_apply_matches_reference_ops(psk, case):
    from conftest import golden_matrix
    from oracle import krylov
    A = golden_matrix(load_golden(case))
    v = np.random.default_rng(2).standard_normal(A.shape[0])
    M = psk.RightIC().form(A)
    assert _rel(M.applyRight(v), krylov.ic_form(A)(v)) <= 1e-12
    assert np.array_equal(M.applyLeft(v), v)


@pytest.mark.parametrize("n,seed", [(1, 0), (37, 1), (2000, 2), (20000, 3), (50000, 4)])
def test_trisolve_chain_random(psk, n, seed):
    """out = (U^-1 L^-1 v[gin])[gout] for random unit/non-unit factors (rows of 0..40 entries)."""
    from pysolvers_amd.Linear import TriangularSolveChain
    rng = np.random.default_rng(seed)
    dens = min(1.0, (8.0 if seed < 4 else 3.0) / max(n, 1))   # seed 4: short rows -> band-eligible
    Lo = sp.tril(sp.random(n, n, density=dens, random_state=rng), k=-1).tocsr() * 0.1
    Up = sp.triu(sp.random(n, n, density=dens, random_state=rng), k=1).tocsr() * 0.1
    dl, du = 1.0 + rng.random(n), 1.0 + rng.random(n)
    gin, gout = rng.permutation(n), rng.permutation(n)
    v = rng.standard_normal(n)
    for l_unit, u_unit in ((True, False), (False, True), (False, False)):
        L = (Lo + sp.diags(dl)).tocsr()
        U = (Up + sp.diags(du)).tocsr()
        Ld = (Lo + sp.eye(n)).tocsr() if l_unit else L
        Ud = (Up + sp.eye(n)).tocsr() if u_unit else U
        ref = spla.spsolve_triangular(Ud, spla.spsolve_triangular(Ld, v[gin], lower=True), lower=False)[gout]
        M = TriangularSolveChain(n, L=L, l_unit=l_unit, U=U, u_unit=u_unit, gather_in=gin, gather_out=gout)
        assert _rel(M.apply(v), ref) <= 1e-12
        for sched in ("syncfree", "band", "lds"):            # every schedule, forced where eligible
            for f in ("L", "U"):
                if sched == "syncfree" or (sched == "band" and M.schedule(f)["est_band_us"] >= 0) or \
                        (sched == "lds" and n <= 18432):
                    M.schedule(f, set=sched)
            assert _rel(M.apply(v), ref) <= 1e-12, sched
    # single factors, no permutations
    M = TriangularSolveChain(n, U=U)
    assert _rel(M.apply(v), spla.spsolve_triangular(U, v, lower=False)) <= 1e-12
    M = TriangularSolveChain(n, L=L)
    assert _rel(M.apply(v), spla.spsolve_triangular(L, v, lower=True)) <= 1e-12
    info = M.device_info()
    assert info["n"] == n and info["nnz_u"] == 0 and info["levels_l"] >= 1


def test_trisolve_rejects_bad_factors(psk):
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear import TriangularSolveChain
    U = sp.csr_matrix(np.array([[1.0, 0.0], [2.0, 1.0]]))       # entry below the diagonal
    with pytest.raises(N.PskError):
        TriangularSolveChain(2, U=U)
    L = sp.csr_matrix(np.array([[0.0, 0.0], [2.0, 1.0]]))       # missing diagonal, non-unit
    L.eliminate_zeros()
    with pytest.raises(N.PskError):
        TriangularSolveChain(2, L=L)
    with pytest.raises(N.PskError):
        TriangularSolveChain(2, L=L, l_unit=True, gather_in=np.array([0, 0]))   # not a permutation


def test_gauss_seidel_narrow_band_large(psk, monkeypatch):
    """FD 1024^2 triu: 256 blocks of 4 grid lines, 32 staged chunks each — the narrow band kernel
    (one solving wave, staging waves re-polling the external snapshots) and the barrier band kernel
    (PSK_BAND_NARROW=0) both match spsolve_triangular, and each other bit for bit."""
    from oracle import fdlap
    from pysolvers_amd.Linear import TriangularSolveChain
    m = 1024
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    U = sp.triu(A).tocsr()
    v = np.random.default_rng(5).standard_normal(A.shape[0])
    ref = spla.spsolve_triangular(U, v, lower=False)
    outs = []
    for narrow in ("1", "0"):
        monkeypatch.setenv("PSK_BAND_NARROW", narrow)
        M = TriangularSolveChain(A.shape[0], U=U)
        M.schedule("U", set="band")
        outs.append(M.apply(v))
        assert _rel(outs[-1], ref) <= 1e-12, narrow
        assert _rel(M.apply(v), ref) <= 1e-12, narrow   # re-apply (sentinel refill)
    assert np.array_equal(outs[0], outs[1])   # same per-row arithmetic in both kernels


@pytest.mark.parametrize("m", [64, 300])
def test_gauss_seidel_factor_schedules(psk, m):
    """triu(-FD2D) (the GS smoother's factor, ClassicSmoothers.py:33): band and sync-free schedules
    both solve it; the band schedule must have an LDS ring (in-block distance m) at these sizes."""
    from oracle import fdlap
    from pysolvers_amd.Linear import TriangularSolveChain
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    U = sp.triu(A).tocsr()
    v = np.random.default_rng(m).standard_normal(A.shape[0])
    ref = spla.spsolve_triangular(U, v, lower=False)
    M = TriangularSolveChain(A.shape[0], U=U)
    info = M.schedule("U")
    assert info["est_band_us"] > 0 and info["est_syncfree_us"] > 0
    outs = {}
    for sched in ("band", "syncfree", "lds") if A.shape[0] <= 18432 else ("band", "syncfree"):
        M.schedule("U", set=sched)
        outs[sched] = M.apply(v)
        assert _rel(outs[sched], ref) <= 1e-12, sched
        assert _rel(M.apply(v), ref) <= 1e-12, sched          # re-apply (sentinel refill)
    if "lds" in outs:   # the LDS schedule runs the sync-free row arithmetic: bit-identical
        assert np.array_equal(outs["lds"], outs["syncfree"])


@pytest.mark.parametrize("n,dens", [(3000, 0.08), (18432, 0.002)])
def test_lds_schedule_matches_syncfree(psk, n, dens):
    """The single-workgroup LDS schedule (x in LDS) on coarse-LU-like factors: long rows (> 3 chunks
    of 64 entries at n=3000) and the largest eligible size. Bit-identical to the sync-free kernel
    (same per-row arithmetic), within 1e-12 of spsolve_triangular; a larger factor is refused."""
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear import TriangularSolveChain
    rng = np.random.default_rng(n)
    Lo = sp.tril(sp.random(n, n, density=dens, random_state=rng), k=-1).tocsr() * (2.0 / (dens * n))
    L = (Lo + sp.diags(1.0 + rng.random(n))).tocsr()
    U = L.T.tocsr()
    v = rng.standard_normal(n)
    ref = spla.spsolve_triangular(U, spla.spsolve_triangular(L, v, lower=True), lower=False)
    M = TriangularSolveChain(n, L=L, U=U)
    outs = {}
    for sched in ("syncfree", "lds"):
        for f in ("L", "U"):
            M.schedule(f, set=sched)
        outs[sched] = M.apply(v)
        assert _rel(outs[sched], ref) <= 1e-12, sched
        assert _rel(M.apply(v), ref) <= 1e-12, sched
    assert np.array_equal(outs["lds"], outs["syncfree"])
    big = TriangularSolveChain(18433, L=sp.eye(18433, format="csr"))
    with pytest.raises(N.PskError):
        big.schedule("L", set="lds")


def _grid_available(M, which):
    from pysolvers_amd import _native as N
    try:
        M.schedule(which, set="grid")
        return True
    except N.PskError:
        return False


@pytest.mark.parametrize("m,lower", [(64, False), (300, False), (1024, False), (300, True)])
def test_grid_schedule_fd_factors(psk, m, lower):
    """The 2-D stencil (grid) schedule on triu(-FD2D) — the Gauss-Seidel smoother's factor
    (ClassicSmoothers.py:33) — and on tril(-FD2D) (forward solve): eligible, within 1e-12 of
    spsolve_triangular, and bit-identical to the band schedule (same per-row arithmetic)."""
    from oracle import fdlap
    from pysolvers_amd.Linear import TriangularSolveChain
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    T = (sp.tril(A) if lower else sp.triu(A)).tocsr()
    v = np.random.default_rng(m).standard_normal(A.shape[0])
    ref = spla.spsolve_triangular(T, v, lower=lower)
    f = "L" if lower else "U"
    M = TriangularSolveChain(A.shape[0], **({"L": T} if lower else {"U": T}))
    assert _grid_available(M, f)
    g = M.apply(v)
    assert _rel(g, ref) <= 1e-12
    assert np.array_equal(M.apply(v), g)                 # re-apply (sentinel refill), deterministic
    M.schedule(f, set="band")
    assert np.array_equal(M.apply(v), g)


def test_grid_schedule_sa_coarse_operator(psk):
    """An SA coarse operator of a 2-D grid (level 3 of the -FD 1024^2 hierarchy: 342 x 512 aggregate
    lines, dependencies up to 2 lines back with diagonal neighbours): the grid schedule takes it, and
    matches the band schedule bit for bit and spsolve_triangular to 1e-12; with a permuted input and
    output (the pre-gather path) it matches the same solve done by numpy indexing. Its dependency
    (1 line back, 2 positions ahead) sits on every other line only, so the plan takes the half-integer
    skew 5/2 (g(y) = (5y + 1) >> 1: 1620 steps per sweep where the integer skew 3 needs 1874)."""
    from oracle import fdlap
    from pysolvers_amd.Linear import SmoothedAggregationMLHierarchy, TriangularSolveChain
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, 1024)
    h = SmoothedAggregationMLHierarchy(A, numLevels=5)
    A3 = h.matrix(3).tocsr()
    U = sp.triu(A3).tocsr()
    n = A3.shape[0]
    v = np.random.default_rng(3).standard_normal(n)
    ref = spla.spsolve_triangular(U, v, lower=False)
    M = TriangularSolveChain(n, U=U)
    assert _grid_available(M, "U")
    gi = M.grid_info("U")
    assert (gi["w"], gi["sigma2"], gi["phase"]) == (342, 5, 1), gi
    assert gi["dict_records"] > 0
    g = M.apply(v)
    assert _rel(g, ref) <= 1e-12
    M.schedule("U", set="band")
    assert np.array_equal(M.apply(v), g)
    rng = np.random.default_rng(4)
    pin, pout = rng.permutation(n).astype(np.int32), rng.permutation(n).astype(np.int32)
    P = TriangularSolveChain(n, U=U, gather_in=pin, gather_out=pout)
    assert _grid_available(P, "U")
    assert np.array_equal(P.apply(v), M.apply(v[pin])[pout])


@functools.lru_cache(maxsize=1)
def _fd2048_sa_levels():
    from oracle import fdlap
    from pysolvers_amd.Linear import SmoothedAggregationMLHierarchy
    h = SmoothedAggregationMLHierarchy(-fdlap.fd_laplacian_2d(-1.0, 1.0, 2048), numLevels=5)
    return {lev: h.matrix(lev).tocsr() for lev in (2, 3)}


@pytest.mark.parametrize("level,lower", [(3, False), (3, True), (2, False), (2, True)])
def test_grid_half_skew_sa_levels(psk, monkeypatch, level, lower):
    """SA levels 3 and 2 of the -FD 2048^2 hierarchy (1024 x 683 and 342 x 228 aggregate lines) take
    the half-integer skew 3/2 (their dependencies 1 line back and 1 ahead sit on every other line),
    upper and lower factors: within 1e-12 of spsolve_triangular, and bit-identical to the band
    schedule and to the grid schedule's per-step records (no dictionary)."""
    from pysolvers_amd.Linear import TriangularSolveChain
    Al = _fd2048_sa_levels()[level]
    T = (sp.tril(Al) if lower else sp.triu(Al)).tocsr()
    n = Al.shape[0]
    f = "L" if lower else "U"
    v = np.random.default_rng(level).standard_normal(n)
    ref = spla.spsolve_triangular(T, v, lower=lower)
    outs = []
    for dict_on in ("1", "0"):
        monkeypatch.setenv("PSK_TRISOLVE_GRID_DICT", dict_on)
        M = TriangularSolveChain(n, **({"L": T} if lower else {"U": T}))
        assert _grid_available(M, f)
        gi = M.grid_info(f)
        assert gi["sigma2"] % 2 == 1, gi
        assert (gi["dict_records"] > 0) == (dict_on == "1"), gi
        outs.append(M.apply(v))
        assert np.array_equal(M.apply(v), outs[-1])      # re-apply (sentinel refill), deterministic
    assert np.array_equal(outs[0], outs[1])
    assert _rel(outs[0], ref) <= 1e-12
    M.schedule(f, set="band")
    assert np.array_equal(M.apply(v), outs[0])


@pytest.mark.parametrize("m,lower", [(300, False), (300, True), (1024, False)])
def test_grid_record_dictionary_bitwise(psk, monkeypatch, m, lower):
    """The grid schedule's record dictionary (one index per lane-step into an LDS table of the
    distinct records; FD factors have a handful) gives the same bits as streaming the records."""
    from oracle import fdlap
    from pysolvers_amd.Linear import TriangularSolveChain
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    T = (sp.tril(A) if lower else sp.triu(A)).tocsr()
    v = np.random.default_rng(m + 7).standard_normal(A.shape[0])
    f = "L" if lower else "U"
    outs = []
    for dict_on in ("1", "0"):
        monkeypatch.setenv("PSK_TRISOLVE_GRID_DICT", dict_on)
        M = TriangularSolveChain(A.shape[0], **({"L": T} if lower else {"U": T}))
        assert _grid_available(M, f)
        outs.append(M.apply(v))
    assert np.array_equal(outs[0], outs[1])
    ref = spla.spsolve_triangular(T, v, lower=lower)
    assert _rel(outs[0], ref) <= 1e-12


@pytest.mark.parametrize("lower", [False, True])
def test_grid_schedule_partial_line(psk, lower):
    """A 9-point stencil on lines of w = 300 whose LAST natural line is partial (n = 300*180 + 77): the
    upper factor's solve order then STARTS with the partial line (the shape of SA level 2 of -FD
    8192^2: 1365 lines of 911 after one of 228), which the grid schedule takes with a leading offset
    of w - n mod w empty positions; the lower factor ends with it. Within 1e-12 of
    spsolve_triangular and bit-identical to the band schedule."""
    from pysolvers_amd.Linear import TriangularSolveChain
    w, n = 300, 300 * 180 + 77
    q = np.arange(n)
    y, x = q // w, q % w
    rows, cols = [], []
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dy == 0 and dx == 0:
                continue
            yy, xx = y + dy, x + dx
            ok = (xx >= 0) & (xx < w) & (yy >= 0) & (yy * w + xx < n)
            rows.append(q[ok])
            cols.append((yy * w + xx)[ok])
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    A = sp.csr_matrix((np.full(len(rows), -1.0), (rows, cols)), shape=(n, n)) + sp.diags(np.full(n, 8.5))
    T = (sp.tril(A) if lower else sp.triu(A)).tocsr()
    v = np.random.default_rng(5).standard_normal(n)
    ref = spla.spsolve_triangular(T, v, lower=lower)
    f = "L" if lower else "U"
    M = TriangularSolveChain(n, **({"L": T} if lower else {"U": T}))
    assert _grid_available(M, f)
    g = M.apply(v)
    assert _rel(g, ref) <= 1e-12
    assert np.array_equal(M.apply(v), g)
    M.schedule(f, set="band")
    assert np.array_equal(M.apply(v), g)


@pytest.mark.parametrize("scale", [1e-280, 1e280])
def test_grid_markstein_range_fallback(psk, scale):
    """The grid dictionary kernel divides by a Markstein correction from RN(1/d), exact while the
    right-hand side stays in [2^-900, 2^901); a step outside it flags the launch and a conditional
    pass re-solves with the IEEE division. A right-hand side scaled far outside the range must still
    give the band schedule's (IEEE) bits, and the flag must be cleared for the next, in-range apply."""
    from oracle import fdlap
    from pysolvers_amd.Linear import TriangularSolveChain
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, 300)
    T = sp.triu(A).tocsr()
    n = A.shape[0]
    M = TriangularSolveChain(n, U=T)
    assert _grid_available(M, "U")
    v = np.random.default_rng(9).standard_normal(n)
    vs = v * scale
    g_small, g = M.apply(vs), M.apply(v)
    M.schedule("U", set="band")
    assert np.array_equal(M.apply(vs), g_small)
    assert np.array_equal(M.apply(v), g)
    ref = spla.spsolve_triangular(T, vs, lower=False)
    assert np.all(np.isfinite(g_small)) and _rel(g_small / scale, ref / scale) <= 1e-12   # norms would under/overflow


# ---------------------------------------------------------------------------------------------
# dense coarse solve (round 5, pysolvers_amd/csrc/dense.hip): x = A_c^-1 f as one streamed GEMV.
# Bar: within 1e-12 (max-norm, relative) of SuperLU's solve of the same matrix (spsolve, VCycleManager.py:36),
# bitwise reproducible run to run, and the AMG apply with it within 1e-10 of the oracle (above).

def _sa_coarse(m, L):
    from oracle import fdlap
    from pysolvers_amd.Linear.SmoothedAggregation import SmoothedAggregationMLHierarchy
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    return sp.csr_matrix(SmoothedAggregationMLHierarchy(sp.csr_matrix(A), numLevels=L).matrix(0))


def _maxrel(a, b):
    return np.max(np.abs(a - b)) / np.max(np.abs(b))


@pytest.mark.parametrize("m,L,refine", [(64, 2, 0), (384, 3, 0), (2048, 4, 0), (2048, 4, 1)])
def test_dense_coarse_matches_splu(psk, m, L, refine):
    """SA coarse operators of -FD m^2: n_c = 1,024 (one column segment), ~4,800 (three) and 9,715 (five;
    the partial last segment), with and without the refinement step."""
    from pysolvers_amd.Linear.AMGPreconditioner import DenseInverseSolver, coarse_factor
    Ac = _sa_coarse(m, L)
    lu = coarse_factor(Ac)
    D = DenseInverseSolver(Ac, refine=refine)
    rng = np.random.default_rng(m + refine)
    for _ in range(3):
        f = rng.standard_normal(Ac.shape[0])
        x = D.apply(f)
        assert _maxrel(x, lu.solve(f, trans='T')) <= 1e-12
        assert np.array_equal(D.apply(f).view(np.uint64), x.view(np.uint64))


@pytest.mark.parametrize("n,seed", [(1, 0), (7, 1), (2049, 2), (4097, 3)])
def test_dense_inverse_random(psk, n, seed):
    """Odd sizes (row pitch padding, a one-column last segment), nonsymmetric, against numpy's solve."""
    from pysolvers_amd.Linear.AMGPreconditioner import DenseInverseSolver
    rng = np.random.default_rng(seed)
    A = sp.random(n, n, density=min(1.0, 6.0 / n), random_state=rng) + sp.diags(4.0 + rng.random(n))
    A = sp.csr_matrix(A)
    f = rng.standard_normal(n)
    x = DenseInverseSolver(A).apply(f)
    ref = np.linalg.solve(A.toarray(), f)
    assert _maxrel(x, ref) <= 1e-12


def test_dense_inverse_singular_refused(psk):
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear.AMGPreconditioner import DenseInverseSolver
    A = sp.csr_matrix(np.array([[1.0, 2.0], [2.0, 4.0]]))
    with pytest.raises(N.PskError):
        DenseInverseSolver(A)


def test_amg_dense_vs_lu_coarse(psk):
    """The same hierarchy with either coarse solve: applies within 1e-12 of each other, the dense one by
    default."""
    from oracle import fdlap
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, 1024)
    v = np.random.default_rng(4).standard_normal(A.shape[0])
    Md = psk.AMG(numIters=2, numLevels=4).form(A)
    Ml = psk.AMG(numIters=2, numLevels=4, coarse="lu").form(A)
    assert Md.coarse_kind == "dense" and Ml.coarse_kind == "lu"
    assert _rel(Md.applyRight(v), Ml.applyRight(v)) <= 1e-12


# ---------------------------------------------------------------------------------------------
# levels schedule (round 5, ilu.hip sptrsv_levels_kernel): one workgroup, a dependency level per step
# behind a barrier, x in an LDS ring. Bars: bit-identical to the band and grid schedules (the same per-row
# arithmetic: fma over the stored entries in stored order from 0.0, then (b - acc) / d), 1e-12 against
# scipy on random chains with permutations, and the SA level-1 Gauss-Seidel factor it is planned for.

@pytest.mark.parametrize("m", [96, 256])
def test_levels_schedule_matches_band_and_grid_bitwise(psk, monkeypatch, m):
    from oracle import fdlap
    from pysolvers_amd.Linear import TriangularSolveChain
    monkeypatch.setenv("PSK_TRISOLVE_LEVELS", "1")   # build the levels layout at creation
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    U = sp.triu(A).tocsr()
    v = np.random.default_rng(m).standard_normal(A.shape[0])
    M = TriangularSolveChain(A.shape[0], U=U)
    assert M.schedule("U")["schedule"] == "levels"
    y = M.apply(v)
    assert _rel(y, spla.spsolve_triangular(U, v, lower=False)) <= 1e-12
    for sched in ("band", "grid"):
        M.schedule("U", set=sched)
        assert np.array_equal(M.apply(v).view(np.uint64), y.view(np.uint64)), sched
    M.schedule("U", set="levels")
    assert np.array_equal(M.apply(v).view(np.uint64), y.view(np.uint64))   # run to run


@pytest.mark.parametrize("n,seed", [(1, 0), (37, 1), (2000, 2), (20000, 5)])
def test_levels_schedule_random_chain(psk, monkeypatch, n, seed):
    """Random unit / non-unit factors with gather permutations (the ILU chain's shape), rows of 0..16
    entries, forced onto the levels schedule."""
    from pysolvers_amd.Linear import TriangularSolveChain
    monkeypatch.setenv("PSK_TRISOLVE_LEVELS", "1")
    rng = np.random.default_rng(seed)
    dens = min(1.0, 4.0 / max(n, 1))
    Lo = sp.tril(sp.random(n, n, density=dens, random_state=rng), k=-1).tocsr() * 0.1
    Up = sp.triu(sp.random(n, n, density=dens, random_state=rng), k=1).tocsr() * 0.1
    dl, du = 1.0 + rng.random(n), 1.0 + rng.random(n)
    gin, gout = rng.permutation(n), rng.permutation(n)
    v = rng.standard_normal(n)
    for l_unit, u_unit in ((True, False), (False, True), (False, False)):
        L = (Lo + sp.diags(dl)).tocsr()
        U = (Up + sp.diags(du)).tocsr()
        Ld = (Lo + sp.eye(n)).tocsr() if l_unit else L
        Ud = (Up + sp.eye(n)).tocsr() if u_unit else U
        ref = spla.spsolve_triangular(Ud, spla.spsolve_triangular(Ld, v[gin], lower=True), lower=False)[gout]
        M = TriangularSolveChain(n, L=L, l_unit=l_unit, U=U, u_unit=u_unit, gather_in=gin, gather_out=gout)
        levels_used = [M.schedule(f)["schedule"] == "levels" for f in ("L", "U")]
        assert _rel(M.apply(v), ref) <= 1e-12
        if n <= 2000:   # (larger random factors may reach further back than the 16384-slot ring: not eligible)
            assert all(levels_used)


def test_levels_schedule_sa_level1(psk, monkeypatch):
    """Level 1 of the SA hierarchy of -FD 1024^2 (5 levels, 2167 rows): the Gauss-Seidel factor triu(A_1)
    is the kind the levels schedule is planned for (at -FD 8192^2: 131k rows, 1706 levels; narrow levels,
    dependencies a bounded number of positions back); forced, against the sync-free schedule (lane-tree
    row sums: not bitwise) and scipy."""
    from pysolvers_amd.Linear import TriangularSolveChain
    monkeypatch.setenv("PSK_TRISOLVE_LEVELS", "1")
    A1 = _sa_level(1024, 5, 1)
    U = sp.triu(A1).tocsr()
    v = np.random.default_rng(3).standard_normal(A1.shape[0])
    M = TriangularSolveChain(A1.shape[0], U=U)
    assert M.schedule("U")["schedule"] == "levels"
    y = M.apply(v)
    assert _rel(y, spla.spsolve_triangular(U, v, lower=False)) <= 1e-12
    M.schedule("U", set="syncfree")
    assert _rel(M.apply(v), y) <= 1e-13


def _sa_level(m, L, k):
    from oracle import fdlap
    from pysolvers_amd.Linear.SmoothedAggregation import SmoothedAggregationMLHierarchy
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    return sp.csr_matrix(SmoothedAggregationMLHierarchy(sp.csr_matrix(A), numLevels=L).matrix(k))
