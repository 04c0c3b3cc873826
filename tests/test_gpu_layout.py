"""The SpMV storage layouts (psk_csr_layout: CSR tiles / 256-row slices / diagonals) give bit-identical
y — and therefore bit-identical solver trajectories — on every SpMV mode the solvers use.

Bar: bit-exact (scipy csr_matvec sums each row in stored order from 0.0 with rounded products;
every layout does exactly that, IterativeLinearSolver.py:94-106).
"""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import case_precond, golden_matrix, load_golden, product_prec_type, solver_cases

from test_gpu_parity import _check_against_golden, _ragged_matrix

pytestmark = pytest.mark.gpu


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


def test_layout_auto_choice(psk, monkeypatch):
    """FD rows lie on 5 diagonals of one value each (diagonal layout chosen; without it: sliced with a
    value dictionary); random ragged rows would pad (CSR kept)."""
    assert psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, 64).layout == "diag"
    # FD 2^2: no row holds all four neighbour diagonals, and one mostly empty slice
    assert psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, 2).layout == "csr"
    monkeypatch.setenv("PSK_SPMV_DIAG", "0")
    assert psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, 64).layout == "sliced_dict"
    monkeypatch.delenv("PSK_SPMV_DIAG")
    rng = np.random.default_rng(5)
    assert psk.DeviceCSR.from_scipy(_ragged_matrix(rng, 5000)).layout == "csr"


@pytest.mark.parametrize("n,long_rows,empty_rows", [
    (1, (), ()), (7, (), (3,)), (257, (), (0, 256)), (5000, (17, 4096), (5, 6, 7)), (70001, (300,), (69999,)),
])
def test_spmv_every_layout_bitwise(psk, n, long_rows, empty_rows):
    """Ragged rows, empty rows, rows longer than the register slots (loop path), partial last slice;
    n <= 32768 packs every slice (16-bit deltas), n = 70001 leaves most slices wide."""
    rng = np.random.default_rng(n + 11)
    A = _ragged_matrix(rng, n, long_rows, empty_rows)
    x = rng.standard_normal(n)
    x[rng.integers(0, n, size=max(1, n // 50))] = -0.0
    ref = A @ x
    dA = psk.DeviceCSR.from_scipy(A)
    for lay in ("sliced", "csr", "sliced_wide", "sliced"):
        slots, packed = dA.set_layout(lay)
        assert dA.layout == lay or (lay == "sliced" and packed == 0 and dA.layout == "sliced_wide")
        if lay != "csr":
            assert slots >= A.nnz
        if lay == "sliced" and n <= 32768:
            assert packed == slots
        if lay == "sliced_wide":
            assert packed == 0
        y = psk.mvmult(dA, x)
        assert np.array_equal(y.view(np.uint64), ref.view(np.uint64)), lay


def test_spmv_mixed_packed_and_wide_slices(psk):
    """A banded matrix with a few far-off entries: the slices holding them stay 32-bit, the rest pack."""
    rng = np.random.default_rng(21)
    n = 100000
    A = sp.diags([rng.standard_normal(n - 300), rng.standard_normal(n), rng.standard_normal(n - 1)], [-300, 0, 1],
                 format="lil")
    for i in (10, 40000, 99999):
        A[i, (i + 50000) % n] = 2.5
        A[i, (i + 32767) % n] = -1.5
    A = A.tocsr()
    x = rng.standard_normal(n)
    dA = psk.DeviceCSR.from_scipy(A)
    assert dA.layout == "sliced"          # random values: no dictionary
    slots, packed = dA.set_layout("sliced")
    assert 0 < packed < slots
    assert np.array_equal(psk.mvmult(dA, x), A @ x)


def test_spmv_rectangular_every_layout(psk):
    """AMG transfer operators are rectangular (x has ncols entries)."""
    rng = np.random.default_rng(3)
    A = sp.random(3000, 700, density=0.004, random_state=4, format="csr")
    x = rng.standard_normal(700)
    dA = psk.DeviceCSR.from_scipy(A, rectangular=True)
    for lay in ("csr", "sliced", "sliced_wide"):
        dA.set_layout(lay)
        assert np.array_equal(psk.mvmult(dA, x), A @ x)


def test_fd_large_layouts_bitwise(psk):
    """FD 3163^2 (the metric's N = 10M): the sliced y equals the C oracle's csr_matvec."""
    from oracle import fdlap, native
    m = 3163
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    assert dA.layout == "diag"
    x = np.random.default_rng(1).random(m * m)
    yd = psk.mvmult(dA, x)
    slots, packed = dA.set_layout("sliced")
    nnz = 5 * m * m - 4 * m
    assert packed == slots and nnz <= slots < nnz + 4 * m + 5 * 256   # all 16-bit; pads: boundary rows, last slice
    ys = psk.mvmult(dA, x)
    ref = native.csr_matvec(fdlap.fd_laplacian_2d(-1.0, 1.0, m), x)
    assert np.array_equal(ys, ref)
    assert np.array_equal(yd, ref)
    for lay in ("csr", "sliced_wide", "sliced_dict", "diag"):
        dA.set_layout(lay)
        assert dA.layout == lay
        assert np.array_equal(psk.mvmult(dA, x), ref)


def _solve_case(psk, case, d, monkeypatch, layout):
    """The golden case solved with every matrix (A and any AMG hierarchy operator) in `layout`."""
    monkeypatch.setenv("PSK_SPMV_LAYOUT", layout)
    ctl = _ctl(maxiter=case["maxiter"], tau=case["tau"], failOnMaxiter=bool(case["fail_on_maxiter"]))
    f = psk.PCG if case["kind"] == "pcg" else psk.GMRES
    return f(control=ctl, precond=product_prec_type(psk, case_precond(case))).makeSolver().solve(golden_matrix(d),
                                                                                                 d["b"])


@pytest.mark.parametrize("layout", ["csr", "sliced", "sliced_wide", "sliced_dict", "diag"])
@pytest.mark.parametrize("case", solver_cases(), ids=lambda c: c["file"][:-4])
def test_solver_matches_reference_each_layout(psk, case, layout, monkeypatch):
    """Every golden solver case meets the parity bar with either layout forced everywhere. (The dot
    products fused into the SpMV are summed per workgroup, so where a CSR tile is not 256 rows — DH
    matrices, longer rows — the two layouts round p.Ap differently, like any other reduction order.)"""
    d = load_golden(case["file"])
    _check_against_golden(_solve_case(psk, case, d, monkeypatch, layout), d, case)


@pytest.mark.parametrize("file", ["pcg_fd64_jacobi.npz", "pcg_fd128_jacobi.npz", "pcg_fd32_identity.npz",
                                  "gmres_fd16_identity.npz", "gmres_fd32_jacobi.npz", "gmres_fd32_ilut.npz"])
def test_fd_trajectories_bitwise_across_layouts(psk, file, monkeypatch):
    """FD rows: a CSR tile is 256 rows, exactly one slice, so even the fused dot products (kSpmvDot,
    kSpmvPlainDot, kSpmvJacobiDot, kSpmvResid) are summed in the same order: identical bits."""
    case = next(c for c in solver_cases() if c["file"] == file)
    d = load_golden(file)
    s1 = _solve_case(psk, case, d, monkeypatch, "csr")
    for lay in ("sliced", "sliced_wide", "sliced_dict", "diag"):
        s2 = _solve_case(psk, case, d, monkeypatch, lay)
        assert s1.iters() == s2.iters() and s1.success() == s2.success()
        assert np.array_equal(s1.soln(), s2.soln())
        assert np.array_equal(s1.info["hist"], s2.info["hist"])


def test_amg_identical_across_layouts(psk, monkeypatch):
    """AMG hierarchy operators (kSpmvResid, kSpmvPlain on R, kSpmvAdd on P) built under each layout."""
    d = load_golden("pcg_negfd32_ic.npz")
    A = golden_matrix(d)
    out = []
    for lay in ("csr", "sliced", "sliced_wide", "sliced_dict", "diag"):
        monkeypatch.setenv("PSK_SPMV_LAYOUT", lay)
        st = psk.PCG(control=_ctl(maxiter=200, tau=1e-8), precond=psk.AMG(numIters=2, numLevels=3)).makeSolver() \
            .solve(A, d["b"])
        out.append(st)
    for o in out[1:]:
        assert out[0].iters() == o.iters()
        assert np.array_equal(out[0].soln(), o.soln())
        assert np.array_equal(out[0].info["hist"], o.info["hist"])


def _fd_rows_reference(m, x, rows):
    """csr_matvec of FDLaplacian2D(-1, 1, m) restricted to `rows`: each row summed from 0.0 in its
    stored order [diag, -m, +m, -1, +1] (absent neighbours skipped), products rounded."""
    h = abs(1.0 - (-1.0)) / float(m + 1)
    dval, oval = -4.0 / h / h, 1.0 / h / h
    ix, iy = rows % m, rows // m
    s = 0.0 + dval * x[rows]
    for ok, off in ((iy > 0, -m), (iy < m - 1, m), (ix > 0, -1), (ix < m - 1, 1)):
        nb = np.where(ok, rows + off, rows)
        s = np.where(ok, s + oval * x[nb], s)
    return s


def test_fd16384_spmv_full_size(psk):
    """configs[3]'s matrix (n = 268M) on one GPU: the default sliced SpMV equals the CSR-layout kernel
    bit for bit over all rows, and both equal csr_matvec on 400k sampled rows plus every boundary row."""
    m = 16384
    n = m * m
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    assert dA.layout == "diag"
    x = np.random.default_rng(12345).random(n)
    y = psk.mvmult(dA, x)
    rng = np.random.default_rng(2)
    edge = np.arange(m, dtype=np.int64)
    rows = np.unique(np.concatenate([rng.integers(0, n, 400_000), edge, n - m + edge, edge * m, edge * m + m - 1]))
    assert np.array_equal(y[rows], _fd_rows_reference(m, x, rows))
    for lay in ("csr", "sliced_dict"):
        dA.set_layout(lay)
        assert np.array_equal(psk.mvmult(dA, x), y), lay


@pytest.mark.parametrize("nvals", [1, 2, 3, 4, 5, 8, 9])
def test_value_dictionary(psk, nvals):
    """Ragged rows (register and loop paths, empty rows, partial last slice) whose values come from
    `nvals` distinct doubles, including -0.0 next to +0.0 and a subnormal: up to 8 (every select-tree
    size class: 2, 4, 8) the auto layout indexes them through a dictionary and y equals scipy bit for
    bit; at 9 there is no dictionary and forcing one fails."""
    from pysolvers_amd import _native as N
    rng = np.random.default_rng(nvals)
    n = 20000
    A = _ragged_matrix(rng, n, (17, 4096), (5, 6, 7))
    pool = np.concatenate([[-0.0, 0.0, 5e-324, 1.0, -1.0 / 3.0], rng.standard_normal(64)])[:nvals]
    A.data = pool[rng.integers(0, nvals, size=A.nnz)]
    x = rng.standard_normal(n)
    ref = A @ x
    dA = psk.DeviceCSR.from_scipy(A)
    if nvals <= 8:
        assert dA.layout in ("csr", "sliced_dict")   # auto: whichever streams fewer bytes
        dA.set_layout("sliced_dict")
        assert dA.layout == "sliced_dict"
        assert np.array_equal(psk.mvmult(dA, x).view(np.uint64), ref.view(np.uint64))
        dA.set_layout("sliced")
        assert dA.layout == "sliced"
        assert np.array_equal(psk.mvmult(dA, x).view(np.uint64), ref.view(np.uint64))
    else:
        with pytest.raises(N.PskError):
            dA.set_layout("sliced_dict")
        assert dA.layout == "csr"        # a failed switch leaves no sliced copy
        assert np.array_equal(psk.mvmult(dA, x), ref)


def test_uniform_jacobi_diagonal(psk, monkeypatch):
    """A constant diagonal (FD) makes DInv one scalar the PCG kernels read instead of a stream: the
    trajectory is bit-identical to the streamed DInv (PSK_JACOBI_UNIFORM=0); a varying diagonal keeps
    the stream."""
    import ctypes
    from pysolvers_amd import _native as N
    from oracle import fdlap
    m = 128
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    varied = (A + sp.diags(np.arange(m * m) * 1e-3)).tocsr()        # a non-constant diagonal
    for mat, expect in ((dA, 1), (psk.DeviceCSR.from_scipy(varied), 0)):
        M = ctypes.c_void_p()
        N.check(N.lib.psk_prec_create(mat.handle, N.PSK_PREC_JACOBI, ctypes.byref(M)), "psk_prec_create")
        u, v = N.I32(), ctypes.c_double()
        N.check(N.lib.psk_prec_jacobi_uniform(M, ctypes.byref(u), ctypes.byref(v)), "psk_prec_jacobi_uniform")
        N.lib.psk_prec_destroy(M)
        assert u.value == expect
        if expect:
            assert v.value == 1.0 / A.diagonal()[0]
    b = A @ np.random.default_rng(3).random(m * m)
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("PSK_JACOBI_UNIFORM", flag)
        st = psk.PCG(control=_ctl(maxiter=2000, tau=1e-10), precond=psk.Jacobi()).makeSolver().solve(dA, b)
        assert st.success()
        out.append(st)
    assert out[0].iters() == out[1].iters()
    assert np.array_equal(out[0].soln(), out[1].soln())
    assert np.array_equal(out[0].info["hist"], out[1].info["hist"])


def _lap3d(k):
    """7-point Laplacian on a k^3 grid, rows stored [diag, -1, +1, -k, +k, -k^2, +k^2] minus the absent ones."""
    n = k ** 3
    idx = np.arange(n)
    ix, iy, iz = idx % k, (idx // k) % k, idx // (k * k)
    rows, cols, vals = [idx], [idx], [np.full(n, 6.0)]
    for ok, off in ((ix > 0, -1), (ix < k - 1, 1), (iy > 0, -k), (iy < k - 1, k), (iz > 0, -k * k), (iz < k - 1, k * k)):
        rows.append(idx[ok])
        cols.append(idx[ok] + off)
        vals.append(np.full(int(ok.sum()), -1.0))
    r, c, v = np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)
    order = np.lexsort((np.concatenate([np.full(len(x), i) for i, x in enumerate(rows)]), r))   # stored order
    indptr = np.concatenate([[0], np.cumsum(np.bincount(r, minlength=n))])
    return sp.csr_matrix((v[order], c[order], indptr), shape=(n, n))


@pytest.mark.parametrize("which", ["lap3d", "fd_sorted", "tridiag", "rect"])
def test_diag_layout_bitwise(psk, which):
    """The diagonal layout on other constant-coefficient matrices: a 3-D 7-point Laplacian (7 diagonals),
    the FD matrix with sorted column indices (another diagonal order), a tridiagonal (3), and a
    rectangular banded operator (columns past the last row); every SpMV mode the solvers use is exercised
    through mvmult and a solve. y and the trajectories equal the sliced/CSR layouts bit for bit."""
    from oracle import fdlap
    rng = np.random.default_rng(7)
    if which == "lap3d":
        A = _lap3d(40)
    elif which == "fd_sorted":
        A = fdlap.fd_laplacian_2d(-1.0, 1.0, 150).sorted_indices()
    elif which == "tridiag":
        n = 100003
        A = sp.diags([np.full(n - 1, -1.0), np.full(n, 2.5), np.full(n - 1, -1.0)], [-1, 0, 1], format="csr")
    else:
        n = 70000
        A = sp.diags([np.full(n, 0.5), np.full(n, 0.25)], [0, 3], shape=(n, n + 3), format="csr")
    x = rng.standard_normal(A.shape[1])
    x[rng.integers(0, A.shape[1], 50)] = -0.0
    ref = A @ x
    rect = A.shape[0] != A.shape[1]
    dA = psk.DeviceCSR.from_scipy(A, rectangular=True) if rect else psk.DeviceCSR.from_scipy(A)
    assert dA.layout == "diag"
    assert np.array_equal(psk.mvmult(dA, x).view(np.uint64), ref.view(np.uint64))
    if rect:
        return
    b = A @ rng.random(A.shape[0])
    sols = {}
    for lay in ("diag", "sliced_dict", "csr"):
        dA.set_layout(lay)
        sols[lay] = []
        for f, pre in ((psk.PCG, psk.Jacobi()), (psk.GMRES, psk.Jacobi()), (psk.GMRES, None)):
            kw = {"precond": pre} if pre is not None else {}
            sols[lay].append(f(control=_ctl(maxiter=60, tau=1e-9), **kw).makeSolver().solve(dA, b))
    for d, s, c in zip(sols["diag"], sols["sliced_dict"], sols["csr"]):
        # the sliced layout sums the fused dot products over the same 256-row slices: identical bits; the
        # CSR kernel's tiles are 128 rows when rows are long (lap3d), so its dots round differently
        assert d.iters() == s.iters() == c.iters()
        assert np.array_equal(d.soln(), s.soln()) and np.array_equal(d.info["hist"], s.info["hist"])
        assert np.max(np.abs(d.soln() - c.soln())) <= 1e-10 * np.max(np.abs(c.soln()))


def test_diag_layout_refused(psk):
    """No diagonal layout when one entry breaks the rule (a value off its diagonal's, entries off the
    template row's diagonals, a row storing its diagonals in another order): auto keeps the sliced layout,
    forcing fails and leaves the layout as it was."""
    from pysolvers_amd import _native as N
    from oracle import fdlap
    base = fdlap.fd_laplacian_2d(-1.0, 1.0, 40)
    x = np.random.default_rng(3).standard_normal(base.shape[0])
    for how in ("value", "offdiag", "order"):
        A = base.copy().tolil() if how == "offdiag" else base.copy()
        if how == "value":
            A.data[A.indptr[700] + 1] *= 1.0000000000000002
        elif how == "offdiag":   # two rows with entries on two different extra diagonals (33 and 50)
            A[700, 733] = -1.0
            A[900, 950] = -1.0
            A = A.tocsr()
        else:
            s0 = A.indptr[700]
            A.indices[s0:s0 + 5] = A.indices[s0:s0 + 5][::-1].copy()
            A.data[s0:s0 + 5] = A.data[s0:s0 + 5][::-1].copy()
        dA = psk.DeviceCSR.from_scipy(A)
        assert dA.layout != "diag", how
        before = dA.layout
        with pytest.raises(N.PskError):
            dA.set_layout("diag")
        assert dA.layout == before
        assert np.array_equal(psk.mvmult(dA, x), A @ x)


@pytest.mark.parametrize("prec", ["jacobi", "identity"])
def test_pcg_init_edges_diag_vs_csr(psk, prec, monkeypatch):
    """The PCG init fused into the first SpMV (diagonal layout, spmv.hip pcg_init_diag_kernel) against
    pcg_init_kernel + the CSR SpMV, at the init's edges: b = 0 (PCGSolver.py:87-88, converged before any
    iteration), maxiter 0, 1 and 2 (the loop stops before, at and right after the fused launch's first
    consumer), a 1-line grid and a grid smaller than one 256-row tile: identical status, x and history."""
    from oracle import fdlap
    cases = []
    for m in (1, 2, 9, 64):
        A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
        b = A @ np.random.default_rng(m).random(m * m)
        cases += [(A, b, k) for k in (0, 1, 2, 30)] + [(A, np.zeros(m * m), 5)]
    for A, b, k in cases:
        out = []
        for lay in ("csr", "diag"):
            monkeypatch.setenv("PSK_SPMV_LAYOUT", lay)
            ctl = _ctl(maxiter=k, tau=1e-10, failOnMaxiter=False)
            pre = psk.Jacobi() if prec == "jacobi" else psk.IdentityPreconditionerType()
            st = psk.PCG(control=ctl, precond=pre).makeSolver().solve(A, b)
            h = st.info.get("hist")   # absent where the reference reports no iteration (b = 0, maxiter 0)
            out.append((st.iters(), bool(st.success()), st.soln(), None if h is None else np.asarray(h)))
        (i1, s1, x1, h1), (i2, s2, x2, h2) = out
        assert (i1, s1) == (i2, s2), (A.shape, k)
        assert np.array_equal(x1, x2), (A.shape, k)
        assert (h1 is None) == (h2 is None) and (h1 is None or np.array_equal(h1, h2)), (A.shape, k)


def test_fd_pair_kernel_two_level_sums(psk, monkeypatch):
    """The pair-row diagonal kernel (spmv_diagp_kernel: two contiguous rows per lane, 16-B accesses) at a size
    whose fused dot products take the two-level gridsum (1887 tiles, odd n, odd line length): PCG+Jacobi
    (kSpmvDot), GMRES+Jacobi (kSpmvJacobiDot, kSpmvPlainDot, kSpmvResid) and PCG with no preconditioner give the
    CSR layout's trajectories bit for bit — the kernel's wave totals follow wave_total's operand pairs."""
    from oracle import fdlap
    m = 695
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    b = A @ np.random.default_rng(17).random(m * m)
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    assert dA.layout == "diag"
    runs = {}
    for lay in ("diag", "csr"):
        dA.set_layout(lay)
        runs[lay] = [
            psk.PCG(control=_ctl(maxiter=60, tau=0.0, failOnMaxiter=False), precond=psk.Jacobi()).makeSolver()
            .solve(dA, b),
            psk.PCG(control=_ctl(maxiter=45, tau=0.0, failOnMaxiter=False)).makeSolver().solve(dA, b),
            psk.GMRES(control=_ctl(maxiter=25, tau=1e-30, failOnMaxiter=False), precond=psk.Jacobi()).makeSolver()
            .solve(dA, b),
        ]
    for d, c in zip(runs["diag"], runs["csr"]):
        assert d.iters() == c.iters() and d.success() == c.success()
        assert np.array_equal(d.soln(), c.soln())
        assert np.array_equal(d.info["hist"], c.info["hist"])
