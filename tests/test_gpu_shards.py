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
