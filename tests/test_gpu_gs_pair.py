"""The AMG smoother's paired Gauss-Seidel sweeps (round 6, amg.hip gs_pair_kernel) against the serialized
sweeps: two sweeps x <- x + triu(A)^-1 (f - A x) (ClassicSmoothers.py:31-36) in one launch on 5-point grid
levels. Bar: BITWISE equality of the AMG apply with pairing on and off (psk_lab_amg_gs_pair switches it), on
square and rectangular grids whose band split (63 lines per band) leaves full, partial and one-line bands,
with an odd sweep count (a pair plus one serialized sweep), and on the whole -FD 2048^2 five-level apply
(whose serialized path test_gpu_configs pins to the oracle). The pair forms U's off-diagonal sum the way the
factor's schedule does (the grid / band / levels fma chain, or the sync-free / LDS lane partials), so the
equality is checked under each schedule with inexact products (the reference's -FD values). Levels that do
not qualify keep the serialized path: a stencil with one value per diagonal broken, or a coupling removed.
"""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def psk():
    import pysolvers_amd
    return pysolvers_amd


@pytest.fixture(scope="module")
def lab():
    from pysolvers_amd import _native as N
    return N.load_lab(), N


def grid5(m, H, c=(-1.0, 4.0, -1.0), r=(-1.0, -1.0)):
    """5-point operator on an m x H grid (row i = iy * m + ix): kron(I_H, T_m) + kron(T_H, I_m), stored in
    column order per row, one value per diagonal."""
    Tm = sp.diags([c[0], c[1] / 2, c[2]], [-1, 0, 1], shape=(m, m))
    TH = sp.diags([r[0], c[1] / 2, r[1]], [-1, 0, 1], shape=(H, H))
    A = (sp.kron(sp.identity(H), Tm) + sp.kron(TH, sp.identity(m))).tocsr()
    A.eliminate_zeros()   # kron of small blocks stores explicit zeros
    A.sort_indices()
    return A


def pair(lab, M, set_):
    L, N = lab
    on, el = ctypes.c_int32(), ctypes.c_int32()
    N.check(L.psk_lab_amg_gs_pair(M.device_handle, set_, ctypes.byref(on), ctypes.byref(el)), "psk_lab_amg_gs_pair")
    return on.value, el.value


def on_off(psk, lab, A, v, **kw):
    M = psk.AMG(**kw).form(A)
    on, el = pair(lab, M, 1)
    y_on = M.applyRight(v)
    y_dev = M.apply(psk.DeviceVector.from_numpy(v)).numpy()
    pair(lab, M, 0)
    y_off = M.applyRight(v)
    pair(lab, M, 1)
    return on, el, y_on, y_dev, y_off


@pytest.mark.parametrize("m,H", [(128, 128), (64, 63), (300, 127), (700, 64), (5, 400), (1024, 1024)])
def test_gs_pair_bitwise_vs_serialized(psk, lab, m, H):
    A = grid5(m, H)
    v = np.random.default_rng(m * 7 + H).standard_normal(A.shape[0])
    on, el, y_on, y_dev, y_off = on_off(psk, lab, A, v, numIters=2, numLevels=2)
    assert el == 1 and on == 1, (on, el)
    assert np.all(np.isfinite(y_on))
    assert np.array_equal(y_on, y_off)
    assert np.array_equal(y_dev, y_off)


def test_gs_pair_odd_sweeps_and_nonsymmetric(psk, lab):
    """nuPre = 3 (one pair + one serialized sweep), nuPost = 1 (serialized only); unequal couplings."""
    A = grid5(257, 190, c=(-1.25, 4.5, -0.75), r=(-0.5, -1.5))
    v = np.random.default_rng(5).standard_normal(A.shape[0])
    on, el, y_on, y_dev, y_off = on_off(psk, lab, A, v, numIters=2, numLevels=2, nuPre=3, nuPost=1)
    assert el == 1
    assert np.array_equal(y_on, y_off)


def test_gs_pair_negfd_2048_five_levels(psk, lab):
    from oracle import fdlap
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, 2048)
    v = np.random.default_rng(11).standard_normal(A.shape[0])
    on, el, y_on, y_dev, y_off = on_off(psk, lab, A, v, numIters=2, numLevels=5)
    assert el == 1   # the fine level; the SA coarse operators are not 5-point grids
    assert np.array_equal(y_on, y_off)


@pytest.mark.parametrize("how", ["value", "coupling"])
def test_gs_pair_not_eligible_keeps_serialized(psk, lab, how):
    A = grid5(96, 80).tolil()
    if how == "value":
        A[1000, 1001] = -1.001          # one value off its diagonal's
    else:
        A[1000, 1001] = 0.0             # a coupling removed (and its mirror): presence no longer the grid's
        A[1001, 1000] = 0.0
    A = A.tocsr()
    A.eliminate_zeros()
    A.sort_indices()
    v = np.random.default_rng(2).standard_normal(A.shape[0])
    M = psk.AMG(numIters=2, numLevels=2).form(A)
    on, el = pair(lab, M, -1)
    assert (on, el) == (0, 0)
    y = M.applyRight(v)
    assert np.all(np.isfinite(y))


@pytest.mark.parametrize("m", [32, 96, 200])
@pytest.mark.parametrize("sched", ["syncfree", "lds", "band", "grid"])
def test_gs_pair_follows_the_schedule_arithmetic(psk, lab, m, sched):
    """-FD m^2 (FDBratu2D.py:15; values 4/h^2, -1/h^2: rounded products) with the fine smoother's schedule
    forced: pairing on == off bitwise under each."""
    from oracle import fdlap
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    v = np.random.default_rng(m).standard_normal(A.shape[0])
    M = psk.AMG(numIters=2, numLevels=2).form(A)
    S = M._S[-1].operator
    try:
        S.schedule("U", set=sched)
    except Exception as e:   # grid: small factors have no grid plan; lds: too large for one workgroup
        pytest.skip("schedule %s not available: %s" % (sched, e))
    assert S.schedule("U")["schedule"] == sched
    on, el = pair(lab, M, 1)
    assert el == 1
    y_on = M.applyRight(v)
    pair(lab, M, 0)
    y_off = M.applyRight(v)
    assert np.array_equal(y_on, y_off)
