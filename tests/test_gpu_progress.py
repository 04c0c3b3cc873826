"""(The psk_lab_* entry points are libpsk_lab.so's, include/psk_lab.h: a library of their own linked against
libpsk.so, round 6.)

Forward progress of the spin-waiting triangular-solve schedules when their grid cannot be co-resident
(ADVICE r4): a co-running kernel (psk_lab_occupy_begin, on a stream of its own) holds part
of the CUs while the solve runs, and is released only BEHIND the solve on the solver's stream — so the
solve has to complete on whatever the occupiers leave. It must, bit-identical to the unloaded solve, with
no expired wait and without the occupiers reaching their time limit.

Before round 5 the sync-free schedule dealt row k to wave k mod W of a grid sized to the device and the
band schedule block b to workgroup b mod g: with part of that grid unable to start, the resident waves
spun on rows nobody would ever solve (ilu.hip "forward progress without co-residency").
Bar: bit-exact against the same factor's solve on an idle device (same schedule, same per-row arithmetic).
"""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def psk():
    import pysolvers_amd
    from pysolvers_amd import _native as N
    assert N.device_count() >= 1, "no GPU visible to libpsk"
    return pysolvers_amd


def _apply_under_occupiers(handle, v, wgs, lds=100 * 1024):
    """psk_prec_apply of device vector v into a device buffer allocated beforehand, beside the occupiers;
    the result read back after they are released. Nothing is freed inside the window: hipFree waits for
    the whole device, the occupiers' stream included, which would make the test wait for them."""
    from pysolvers_amd import _native as N
    out = psk_mod().DeviceVector(v.n)
    N.check(N.load_lab().psk_lab_occupy_begin(wgs, lds, 30.0), "psk_lab_occupy_begin")
    timed_out = N.I32()
    try:
        N.check(N.lib.psk_prec_apply(handle, v.n, v._p, out._p, N.PSK_DEVICE), "psk_prec_apply")
    finally:
        N.check(N.load_lab().psk_lab_occupy_end(ctypes.byref(timed_out)), "psk_lab_occupy_end")
    xcc = (N.I32 * 8)()
    N.check(N.load_lab().psk_lab_occupy_xcc(xcc), "psk_lab_occupy_xcc")
    assert timed_out.value == 0, "the occupiers hit their time limit: the solve waited for them (per XCD %s)" % list(xcc)
    return out.numpy(), list(xcc)


def psk_mod():
    import pysolvers_amd
    return pysolvers_amd


def _workers(handle, which):
    from pysolvers_amd import _native as N
    e, g = N.I32(), N.I32()
    N.check(N.load_lab().psk_lab_trisolve_workers(handle, which, ctypes.byref(e), ctypes.byref(g)), "workers")
    return e.value, g.value


def test_syncfree_ilu_apply_beside_occupiers(psk):
    """RightILUT (the reference's spilu arguments) on FD 384^2, both factors on the sync-free schedule.
    128 occupiers of 16 waves and 100 KiB of LDS each sit on 128 CUs, leaving room for 4 of the 7
    sync-free workgroups per CU there: the grid cannot all start, the enrolled workers deal the rows."""
    from oracle import fdlap
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, 384)
    M = psk.RightILUT().form(psk.DeviceCSR.from_scipy(A))
    from pysolvers_amd import _native as N
    for f in (0, 1):   # 0 = sync-free (psk_prec_trisolve_schedule)
        N.check(N.lib.psk_prec_trisolve_schedule(M.device_handle, f, 0, None, None, None, None, None), "schedule")
    v = psk.DeviceVector.from_numpy(np.random.default_rng(5).standard_normal(A.shape[0]))
    ref = M.applyRight(v).numpy()
    idle = [_workers(M.device_handle, f) for f in (0, 1)]
    out, _ = _apply_under_occupiers(M.device_handle, v, 128)
    busy = [_workers(M.device_handle, f) for f in (0, 1)]
    assert np.array_equal(out.view(np.uint64), ref.view(np.uint64))
    for (ei, g), (eb, g2) in zip(idle, busy):
        assert g == g2 and ei >= g // 2, (ei, g)     # an idle device: (nearly) every workgroup enrolled
        assert 0 < eb < g, (eb, g)                   # beside the occupiers: fewer workers, still solved


@pytest.mark.parametrize("sched,m", [("band", 1024), ("grid", 1024)])
def test_block_schedules_beside_occupiers(psk, sched, m):
    """triu(-FD m^2) — the Gauss-Seidel smoother's factor (ClassicSmoothers.py:33) — on the band
    schedule (blocks of the solve order) and the grid schedule (64-line bands): workgroups draw their
    blocks from a ticket counter until they run out, so a block only ever waits on blocks held by running
    workgroups. The band grid is 2 workgroups per CU; occupiers leave 1 on half the CUs. For the grid
    schedule (one 147-KiB-LDS workgroup per band, 16 bands) the occupiers hold 30 of the 32 CUs of every
    XCD: the 16 workgroups start wherever the two free CUs per XCD are, in any order.
    What this test cannot show, and the lab probe does (profiles/r5_progress_probe.txt): with 31
    occupiers per XCD, 8 grid workgroups solve all 32 bands of -FD 2048^2 between them in 1.7 ms, but the
    LAUNCH completes only when its other 24 workgroups (nothing left to draw) have been dispatched, and
    the dispatcher does not start them on the CUs the first 8 freed while the occupiers hold the rest.
    These occupiers leave only behind the solve, so such a launch would wait for them forever; any
    kernel of a real caller ends, so it is a launch waiting for CUs, not a wait inside the solve."""
    import scipy.sparse.linalg as spla
    from oracle import fdlap
    from pysolvers_amd.Linear import TriangularSolveChain
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    U = sp.triu(A).tocsr()
    v = np.random.default_rng(9).standard_normal(A.shape[0])
    M = TriangularSolveChain(A.shape[0], U=U)
    M.schedule("U", set=sched)
    ref = M.apply(v)
    assert np.max(np.abs(ref - spla.spsolve_triangular(U, v, lower=False))) <= 1e-12 * np.max(np.abs(ref))
    wgs = 128 if sched == "band" else 240
    out, xcc = _apply_under_occupiers(M.device_handle, psk.DeviceVector.from_numpy(v), wgs)
    if sched == "grid":
        assert max(xcc) <= 30, xcc   # every XCD kept two free CUs (the placement the docstring assumes)
    assert np.array_equal(out.view(np.uint64), ref.view(np.uint64))
    assert np.array_equal(M.apply(v).view(np.uint64), ref.view(np.uint64))   # counters re-armed


def test_amg_apply_beside_occupiers(psk):
    """A whole AMG V-cycle (every level's smoother factor on its own schedule, the coarse LU, the
    transfer SpMVs) beside occupiers on half the CUs: same bits as on an idle device."""
    from oracle import fdlap
    A = -fdlap.fd_laplacian_2d(-1.0, 1.0, 512)
    M = psk.AMG(numIters=2, numLevels=4, smoother=psk.GaussSeidelSmoother).form(psk.DeviceCSR.from_scipy(A))
    v = psk.DeviceVector.from_numpy(np.random.default_rng(2).standard_normal(A.shape[0]))
    ref = M.applyRight(v).numpy()
    out, _ = _apply_under_occupiers(M.device_handle, v, 128)
    assert np.array_equal(out.view(np.uint64), ref.view(np.uint64))
