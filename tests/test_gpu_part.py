"""The partitioned triangular-solve schedule (sptrsv_part_kernel, ilu.hip): strips of the natural
index per workgroup, in-strip dependencies through an LDS cache. It runs the sync-free kernel's
per-row arithmetic, so every test checks it bit for bit against the sync-free schedule on the same
factor, and against the host reference solve (SuperLU ILU.solve / spsolve_triangular) to 1e-12.
The layout is built when the cost model picks it or with PSK_TRISOLVE_PART=1 at creation."""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

pytestmark = pytest.mark.gpu

SCHED = {"syncfree": 0, "part": 4}


@pytest.fixture(scope="module")
def psk():
    import pysolvers_amd
    return pysolvers_amd


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _set(h, which, sched):
    """Force (or with sched=None query) the schedule of factor `which` of a device preconditioner."""
    from pysolvers_amd import _native as N
    sc = ctypes.c_int32()
    N.check(N.lib.psk_prec_trisolve_schedule(h, which, -1 if sched is None else SCHED[sched], ctypes.byref(sc),
                                             None, None, None, None), "psk_prec_trisolve_schedule")
    return sc.value


@pytest.mark.parametrize("m", [192, 512])
def test_part_schedule_ilut(psk, monkeypatch, m):
    """RightILUT of FD m^2 (the reference's spilu call, COLAMD order): strips of the original
    equation / unknown index; the apply matches ILU.solve and the sync-free schedule bit for bit."""
    from oracle import fdlap
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    v = np.random.default_rng(m).standard_normal(A.shape[0])
    monkeypatch.setenv("PSK_TRISOLVE_PART", "1")
    M = psk.RightILUT().form(A)
    monkeypatch.delenv("PSK_TRISOLVE_PART")
    h = M.device_handle
    assert _set(h, 0, None) == 4 and _set(h, 1, None) == 4
    ref = M.ILU().solve(v)
    p = M.applyRight(v)
    assert _rel(p, ref) <= 1e-12
    assert np.array_equal(M.applyRight(v), p)        # re-apply: sentinel refill, LDS tags reset
    for f in (0, 1):
        _set(h, f, "syncfree")
    assert np.array_equal(M.applyRight(v), p)
    _set(h, 0, "part")                               # mixed: part L, sync-free U
    assert np.array_equal(M.applyRight(v), p)


def test_part_schedule_random_long_rows(psk, monkeypatch):
    """Random unit-lower / upper factors with permuted input and output and a few rows longer than
    the three register chunks (the kernel's tail loop), n = 50000 (195 rows per strip)."""
    from pysolvers_amd.Linear import TriangularSolveChain
    n = 50000
    rng = np.random.default_rng(7)
    Lo = sp.tril(sp.random(n, n, density=6.0 / n, random_state=rng), k=-1).tolil()
    for r in rng.choice(np.arange(n // 2, n), 20, replace=False):   # long rows: 300-900 entries
        cols = rng.choice(r, min(r, int(rng.integers(300, 900))), replace=False)
        Lo[r, cols] = rng.random(len(cols)) * 1e-3
    Lo = Lo.tocsr() * 0.1
    Up = sp.triu(sp.random(n, n, density=6.0 / n, random_state=rng), k=1).tocsr() * 0.1
    L = (Lo + sp.eye(n)).tocsr()
    U = (Up + sp.diags(1.0 + rng.random(n))).tocsr()
    gin, gout = rng.permutation(n), rng.permutation(n)
    v = rng.standard_normal(n)
    ref = spla.spsolve_triangular(U, spla.spsolve_triangular(L, v[gin], lower=True), lower=False)[gout]
    monkeypatch.setenv("PSK_TRISOLVE_PART", "1")
    M = TriangularSolveChain(n, L=L, l_unit=True, U=U, gather_in=gin, gather_out=gout)
    monkeypatch.delenv("PSK_TRISOLVE_PART")
    assert M.schedule("L")["schedule"] == "part" and M.schedule("U")["schedule"] == "part"
    p = M.apply(v)
    assert _rel(p, ref) <= 1e-12
    for f in ("L", "U"):
        M.schedule(f, set="syncfree")
    assert np.array_equal(M.apply(v), p)


def test_part_schedule_far_local_dependencies(psk, monkeypatch):
    """Strips of 12000 rows whose rows depend on rows 64 and 9000 back in the natural order: the
    second dependency is in the same strip but further than the LDS cache holds (8192 local
    positions), so it is coded as a published-value read; n = 256 * 12000."""
    from pysolvers_amd.Linear import TriangularSolveChain
    n = 256 * 12000
    i = np.arange(n)
    rows = np.concatenate([i[64:], i[9000:]])
    cols = np.concatenate([i[:-64], i[:-9000]])
    vals = np.concatenate([np.full(n - 64, -0.3), np.full(n - 9000, 0.2)])
    L = (sp.csr_matrix((vals, (rows, cols)), shape=(n, n)) + sp.diags(np.full(n, 2.0))).tocsr()
    v = np.random.default_rng(11).standard_normal(n)
    ref = spla.spsolve_triangular(L, v, lower=True)
    monkeypatch.setenv("PSK_TRISOLVE_PART", "1")
    M = TriangularSolveChain(n, L=L)
    monkeypatch.delenv("PSK_TRISOLVE_PART")
    assert M.schedule("L")["schedule"] == "part"
    p = M.apply(v)
    assert _rel(p, ref) <= 1e-12
    M.schedule("L", set="syncfree")
    assert np.array_equal(M.apply(v), p)


def test_part_schedule_refused_without_layout(psk, monkeypatch):
    """A factor whose partitioned layout was not built refuses set='part' (PSK_ERR_UNSUPPORTED)."""
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear import TriangularSolveChain
    monkeypatch.setenv("PSK_TRISOLVE_PART", "0")
    M = TriangularSolveChain(30000, L=sp.eye(30000, format="csr"))
    with pytest.raises(N.PskError):
        M.schedule("L", set="part")
