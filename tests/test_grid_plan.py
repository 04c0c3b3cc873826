"""Host-only checks of the grid triangular-solve plan (psk_trisolve_grid_plan; no GPU): line width,
skew (twice the skew, sigma2, and its phase: row (y, x) runs at step x + ((sigma2*y + phase) >> 1)),
leading offset. The device solves these plans produce are checked against spsolve_triangular and the
band schedule in tests/test_gpu_amg.py."""
import numpy as np
import pytest
import scipy.sparse as sp

from pysolvers_amd.Linear.TriangularSolve import grid_plan


def _stencil(w, H, offsets, skip=None, diag=8.5):
    """Symmetric stencil on H lines of w positions; skip(y, x, dy, dx) drops a coupling."""
    n = w * H
    q = np.arange(n)
    y, x = q // w, q % w
    rows, cols = [], []
    for dy, dx in offsets:
        for sy, sx in ((dy, dx), (-dy, -dx)):
            yy, xx = y + sy, x + sx
            ok = (xx >= 0) & (xx < w) & (yy >= 0) & (yy < H)
            if skip is not None:
                ok &= ~skip(np.minimum(y, yy), sy, sx, x)
            rows.append(q[ok])
            cols.append((yy * w + xx)[ok])
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    A = sp.csr_matrix((np.full(len(rows), -1.0), (rows, cols)), shape=(n, n))
    A.sum_duplicates()
    return A + sp.diags(np.full(n, diag))


@pytest.mark.parametrize("upper", [True, False])
def test_five_point_integer_skew(upper):
    """triu / tril of the 5-point stencil: (0,1), (1,0) back in solve order, skew 1 (sigma2 = 2)."""
    A = _stencil(300, 200, [(0, 1), (1, 0)])
    T = sp.triu(A) if upper else sp.tril(A)
    p = grid_plan(T, upper)
    assert p is not None and (p["w"], p["H"], p["sigma2"], p["phase"], p["off"]) == (300, 200, 2, 0, 0)
    assert p["steps"] == 299 + 63 + 1


@pytest.mark.parametrize("upper", [True, False])
def test_nine_point_keeps_integer_skew(upper):
    """The full 9-point stencil has the (1 line back, 1 ahead) neighbour on EVERY line: skew 2, no half step."""
    A = _stencil(300, 200, [(0, 1), (1, -1), (1, 0), (1, 1)])
    T = sp.triu(A) if upper else sp.tril(A)
    p = grid_plan(T, upper)
    assert p is not None and (p["sigma2"], p["phase"]) == (4, 0)


@pytest.mark.parametrize("upper", [True, False])
def test_alternate_line_neighbour_takes_half_skew(upper):
    """The (1 line back, 1 ahead) neighbour only between lines 2k and 2k+1: skew 3/2 (sigma2 = 3)
    meets it — the shape SA aggregation leaves on its coarse levels."""
    A = _stencil(300, 200, [(0, 1), (1, -1), (1, 0), (1, 1)], skip=lambda ylo, sy, sx, x: (ylo % 2 == 1) & (sy * sx != 0))
    T = sp.triu(A) if upper else sp.tril(A)
    p = grid_plan(T, upper)
    assert p is not None and p["sigma2"] == 3, p
    # every dependency is >= 1 step back under the plan's g
    g = lambda yy: (p["sigma2"] * yy + p["phase"]) >> 1
    T = sp.csr_matrix(T)
    n, w, off = T.shape[0], p["w"], p["off"]
    rows = np.repeat(np.arange(n), np.diff(T.indptr))
    m = T.indices != rows
    pos = (lambda i: n - 1 - i) if upper else (lambda i: i)
    pr, pc = pos(rows[m]) + off, pos(T.indices[m]) + off
    ur = pr % w + g(pr // w)
    uc = pc % w + g(pc // w)
    assert (ur - uc >= 1).all()
    assert p["steps"] == (w - 1) + g(63) - g(0) + 1


def test_sa_coarse_level_half_skew():
    """Level 3 of the -FD 1024^2 SA hierarchy (342 x 512 aggregate lines): skew 5/2, phase 1, both factors."""
    from oracle import fdlap
    from pysolvers_amd.Linear import SmoothedAggregationMLHierarchy
    A3 = SmoothedAggregationMLHierarchy(-fdlap.fd_laplacian_2d(-1.0, 1.0, 1024), numLevels=5).matrix(3).tocsr()
    for upper in (True, False):
        p = grid_plan(sp.triu(A3) if upper else sp.tril(A3), upper)
        assert p is not None and (p["w"], p["sigma2"], p["phase"], p["off"]) == (342, 5, 1, 0), p


def test_not_a_grid():
    """A random sparse factor is not a 2-D stencil: no plan."""
    rng = np.random.default_rng(0)
    n = 8192
    R = sp.random(n, n, density=4.0 / n, random_state=rng, format="csr")
    T = sp.tril(R, k=-1) + sp.eye(n)
    assert grid_plan(T, False) is None
