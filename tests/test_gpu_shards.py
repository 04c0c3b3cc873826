"""Row-block shards built on ONE GPU (dry communicator, no RCCL): every rank's local CSR must equal
the oracle's remapped block bit for bit, and the SpMV on [owned | halo] must reproduce the global
SpMV rows of that rank bit for bit. (The collectives themselves need >= 2 GPUs; the schedule is
covered on CPU by tests/test_dist_gloo.py.)"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,P", [(64, 2), (64, 3), (100, 8), (7, 7)])
def test_fd_shards_match_oracle(m, P):
    from pysolvers_amd import _native as N
    from oracle import dist_pcg, fdlap
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    x = np.random.default_rng(5).standard_normal(m * m)
    y = A @ x
    for r in range(P):
        comm = ctypes.c_void_p()
        N.check(N.lib.psk_comm_init_dry(P, r, ctypes.byref(comm)), "dry comm")
        h = ctypes.c_void_p()
        rb, re = ctypes.c_int64(), ctypes.c_int64()
        N.check(N.lib.psk_csr_create_fd2d_dist(-1.0, 1.0, m, comm, ctypes.byref(h), ctypes.byref(rb),
                                               ctypes.byref(re)), "fd2d_dist")
        plan = N.fd2d_dist_plan(m, P, r)
        assert (rb.value, re.value) == plan[:2]
        ref = dist_pcg.local_block(m, plan)
        nloc, nnz = ctypes.c_int64(), ctypes.c_int64()
        N.check(N.lib.psk_csr_info(h, ctypes.byref(nloc), ctypes.byref(nnz)), "info")
        assert nloc.value == ref.shape[0] and nnz.value == ref.nnz
        ip = np.empty(nloc.value + 1, np.int32)
        ix = np.empty(nnz.value, np.int32)
        dt = np.empty(nnz.value, np.float64)
        N.check(N.lib.psk_csr_download(h, N.ptr(ip), N.ptr(ix), N.ptr(dt)), "download")
        assert np.array_equal(ip, ref.indptr) and np.array_equal(ix, ref.indices) and np.array_equal(dt, ref.data)
        # [owned | halo_lo | halo_hi] from the global x
        rb_, re_, ncols, hlo, hhi = plan
        xe = np.concatenate([x[rb_:re_], x[rb_ - hlo:rb_], x[re_:re_ + hhi]])
        assert xe.shape[0] == ncols
        yl = np.empty(nloc.value)
        N.check(N.lib.psk_spmv(h, N.ptr(xe), N.ptr(yl), N.PSK_HOST), "spmv")
        assert np.array_equal(yl, y[rb_:re_])
        # Jacobi on the shard uses the local diagonal
        M = ctypes.c_void_p()
        N.check(N.lib.psk_prec_create(h, N.PSK_PREC_JACOBI, ctypes.byref(M)), "jacobi")
        v = x[rb_:re_].copy()
        out = np.empty_like(v)
        N.check(N.lib.psk_prec_apply(M, nloc.value, N.ptr(v), N.ptr(out), N.PSK_HOST), "apply")
        assert np.array_equal(out, np.reciprocal(A.diagonal()[rb_:re_]) * v)
        N.lib.psk_prec_destroy(M)
        N.lib.psk_csr_destroy(h)
        N.lib.psk_comm_destroy(comm)


@pytest.mark.parametrize("m", [64, 333])
def test_rccl_single_rank_pcg_matches_unsharded(m):
    """The sharded PCG driver through a real RCCL communicator of one rank (the collectives all run:
    init partial gather, per-iteration allgathers of p.Ap and (r.r, u.r)) must reproduce the
    unsharded solve bit for bit: with P = 1 the rank-order sum is the value itself and the init
    partials are only zero-padded."""
    from pysolvers_amd import _native as N
    n = m * m
    uid = (ctypes.c_uint8 * N.PSK_UNIQUE_ID_BYTES)()
    N.check(N.lib.psk_comm_unique_id(uid), "unique id")
    comm = ctypes.c_void_p()
    N.check(N.lib.psk_comm_init(1, 0, uid, ctypes.byref(comm)), "comm init")
    hs, hu = ctypes.c_void_p(), ctypes.c_void_p()
    rb, re = ctypes.c_int64(), ctypes.c_int64()
    N.check(N.lib.psk_csr_create_fd2d_dist(-1.0, 1.0, m, comm, ctypes.byref(hs), ctypes.byref(rb),
                                           ctypes.byref(re)), "fd2d_dist")
    assert (rb.value, re.value) == (0, n)
    N.check(N.lib.psk_csr_create_fd2d(-1.0, 1.0, m, ctypes.byref(hu)), "fd2d")
    b = np.random.default_rng(7).random(n)
    out = {}
    for name, h in (("sharded", hs), ("unsharded", hu)):
        M = ctypes.c_void_p()
        N.check(N.lib.psk_prec_create(h, N.PSK_PREC_JACOBI, ctypes.byref(M)), "jacobi")
        ctl = N.PskCtl(maxiter=5000, tau=1e-8, fail_on_maxiter=1, restart=0, check_every=0, time_kernels=0)
        res = N.PskResult()
        x = np.empty(n)
        hist = np.zeros(5000)
        N.check(N.lib.psk_pcg(h, M, N.ptr(b), N.ptr(x), ctypes.byref(ctl), ctypes.byref(res), N.ptr(hist),
                              N.PSK_HOST), name)
        out[name] = (res.iters, res.success, x, hist[:res.hist_len].copy())
        N.lib.psk_prec_destroy(M)
    N.lib.psk_csr_destroy(hs)
    N.lib.psk_csr_destroy(hu)
    N.lib.psk_comm_destroy(comm)
    s, u = out["sharded"], out["unsharded"]
    assert s[1] == 1 and u[1] == 1 and s[0] == u[0]
    assert np.array_equal(s[3], u[3]) and np.array_equal(s[2], u[2])


def _general(name):
    from conftest import golden_matrix, load_golden
    from oracle import fdlap
    if name.startswith("fd"):
        return fdlap.fd_laplacian_2d(-1.0, 1.0, int(name[2:]))
    return golden_matrix(load_golden("pcg_%s_identity.npz" % name))


@pytest.mark.parametrize("name,P", [("dh8", 2), ("dh12", 3), ("dh12", 5), ("fd50", 4)])
def test_general_shards_match_oracle(name, P):
    """psk_csr_create_dist on every rank (dry communicator): local CSR, halo columns and halo peer
    lists equal the oracle's plan; the halo pack kernel sends exactly x[send rows]; the SpMV on
    [owned | halo] reproduces the global rows bit for bit."""
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear.Distributed import Communicator, even_row_starts, halo_cols, shard_csr
    from oracle import dist_pcg
    A = _general(name)
    n = A.shape[0]
    rs = even_row_starts(n, P, A.indptr)
    xg = np.random.default_rng(3).standard_normal(n)
    yg = A @ xg
    for r in range(P):
        comm = Communicator(P, r, dry=True)
        S = shard_csr(A, comm, rs)
        pl = dist_pcg.shard_plan(A, rs, r)
        assert (S.row_begin, S.row_end, S.n, S.ncols) == (pl["rb"], pl["re"], pl["nloc"], pl["ncols"])
        ip, ix, dt = S.to_scipy()
        assert np.array_equal(ip, pl["Aloc"].indptr) and np.array_equal(ix, pl["Aloc"].indices)
        assert np.array_equal(dt, pl["Aloc"].data)
        assert np.array_equal(halo_cols(S), pl["halo"])
        npeers = N.I32()
        ranks = np.zeros(P, np.int32)
        sc, rc, ro = np.zeros(P, np.int64), np.zeros(P, np.int64), np.zeros(P, np.int64)
        N.check(N.lib.psk_csr_halo_peers(S.handle, N.ptr(ranks), N.ptr(sc), N.ptr(rc), N.ptr(ro),
                                         ctypes.byref(npeers)), "peers")
        k = npeers.value
        assert list(ranks[:k]) == sorted(pl["send"])
        for j, q in enumerate(ranks[:k]):
            assert sc[j] == len(pl["send"][q]) and (ro[j], rc[j]) == pl["recv"][q]
        # what halo_exchange would send, through the pack kernel
        xl = psk.DeviceVector.from_numpy(xg[pl["rb"]:pl["re"]])
        sent = psk.DeviceVector(max(int(sc[:k].sum()), 1))
        N.check(N.lib.psk_csr_halo_pack(S.handle, xl._p, sent._p), "pack")
        want = np.concatenate([xg[pl["rb"] + pl["send"][q]] for q in ranks[:k]] + [np.zeros(0)])
        assert np.array_equal(sent.numpy()[:want.shape[0]], want)
        xe = np.concatenate([xg[pl["rb"]:pl["re"]], xg[pl["halo"]]])
        yl = np.empty(S.n)
        N.check(N.lib.psk_spmv(S.handle, N.ptr(xe), N.ptr(yl), N.PSK_HOST), "spmv")
        assert np.array_equal(yl, yg[pl["rb"]:pl["re"]])
        del S
        comm.destroy()


@pytest.mark.parametrize("name", ["dh12", "fd96"])
def test_rccl_single_rank_general_shard_pcg(name):
    """shard_csr through a real one-rank RCCL communicator (creation-time list exchange runs) and the
    unchanged solver API: bit-identical to the unsharded solve."""
    import pysolvers_amd as psk
    from pysolvers_amd.Linear.Distributed import Communicator, shard_csr
    A = _general(name)
    b = A @ np.random.default_rng(11).random(A.shape[0])
    comm = Communicator(1, 0, Communicator.unique_id())
    S = shard_csr(A, comm)
    ctl = psk.CommonSolverArgs(maxiter=4000, tau=1e-8, showIters=False, showFinal=False)
    st_s = psk.PCG(control=ctl, precond=psk.Jacobi()).makeSolver().solve(S, b)
    st_u = psk.PCG(control=ctl, precond=psk.Jacobi()).makeSolver().solve(A, b)
    assert st_s.success() and st_u.success() and st_s.iters() == st_u.iters()
    assert np.array_equal(st_s.info["hist"], st_u.info["hist"]) and np.array_equal(st_s.soln(), st_u.soln())
    del S
    comm.destroy()
