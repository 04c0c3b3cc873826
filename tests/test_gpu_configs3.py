"""configs[3] at its own size: PCG + Jacobi on FDLaplacian2D 16384 x 16384 (n = 268,435,456,
nnz = 1,342,111,744), the system the 8-GPU row-sharded run executes (BASELINE.json configs[3];
PCGSolver.py:109-138).

* unsharded on the device vs the oracle (oracle/krylov.pcg over oracle/fdlap.FDStencil, the
  matrix-free restatement pinned bit for bit to csr_matvec on the reference generator's CSR by
  tests/test_oracle_golden.py): b = A x bit-exact, 3 iterations, residual history within 1e-10 ||b||,
  solution within 1e-10 relative;
* the row-sharded path at the same size: P = 2 ranks on this one GPU (host shared-memory transport;
  RCCL refuses two ranks on one device), 5 iterations: every rank holds bit-identical scalars, and
  the histories and the gathered solution match the unsharded device run within 1e-12 relative
  (the sharded dot products are summed per rank and then in rank order, a different — equally
  fixed — order than one grid-wide reduction, so the last bits may differ).
Host memory: ~30 GB (oracle vectors) in this process, ~8 GB per rank; HBM ~55 GB unsharded.
"""
import os
import socket

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

M = 16384
RTOL = 1e-10


def _ctl(psk, k):
    return psk.CommonSolverArgs(maxiter=k, tau=0.0, failOnMaxiter=False, showIters=False, showFinal=False)


@pytest.fixture(scope="module")
def unsharded():
    """The unsharded device run (5 iterations; the oracle check below uses its first 3 through a
    second 3-iteration solve)."""
    import pysolvers_amd as psk
    from oracle import fdlap
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, M)
    x = np.random.default_rng(12345).random(M * M)
    b = psk.mvmult(dA, x)
    S = fdlap.FDStencil(-1.0, 1.0, M)
    assert np.array_equal(b, S @ x)                                   # csr_matvec bit for bit
    del x
    st5 = psk.PCG(control=_ctl(psk, 5), precond=psk.Jacobi()).makeSolver().solve(dA, b)
    st3 = psk.PCG(control=_ctl(psk, 3), precond=psk.Jacobi()).makeSolver().solve(dA, b)
    del dA
    return dict(b=b, hist5=st5.info["hist"], x5=st5.soln(), hist3=st3.info["hist"], x3=st3.soln(),
                it5=st5.iters(), it3=st3.iters())


def test_fd16384_pcg_jacobi_vs_oracle(unsharded):
    from oracle import fdlap, krylov
    S = fdlap.FDStencil(-1.0, 1.0, M)
    b = unsharded["b"]
    ref = krylov.pcg(S, b, maxiter=3, tau=0.0, fail_on_maxiter=False, precond=krylov.jacobi_form(S))
    assert unsharded["it3"] == ref["iters"] == 3
    nb = np.linalg.norm(b)
    assert np.max(np.abs(unsharded["hist3"] - ref["hist"])) <= RTOL * nb
    assert np.linalg.norm(unsharded["x3"] - ref["soln"]) <= RTOL * np.linalg.norm(ref["soln"])


def test_fd16384_true_residual_after_50_iterations(unsharded):
    """Full-size property past the oracle's reach (its 16384^2 iterations take seconds each): after 50
    PCG+Jacobi iterations the recursive residual the loop reports, ||r_50|| (PCGSolver.py:122,125), and
    the true residual of the returned x, ||b - A x_50|| (one device SpMV, bit-exact to csr_matvec), agree
    within 1e-10 ||b||; a wrong or missing x update (the deferred flushes at k = 7, 15, ..., 47 and the
    final catch-up at k = 49) would leave an O(||b||) gap."""
    import pysolvers_amd as psk
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, M)
    b = unsharded["b"]
    st = psk.PCG(control=_ctl(psk, 50), precond=psk.Jacobi()).makeSolver().solve(dA, b)
    assert st.iters() == 50 and len(st.info["hist"]) == 50
    x = st.soln()
    r = b - psk.mvmult(dA, x)
    del dA, x
    nb = np.linalg.norm(b)
    h = st.info["hist"]
    assert h[-1] < 0.5 * nb                                           # the iteration made progress
    assert abs(np.linalg.norm(r) - h[-1]) <= RTOL * nb


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, REPO)
    import torch.distributed as dist
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear.Distributed import Communicator, fd_laplacian_2d_sharded
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    N.check(N.lib.psk_set_device(0), "psk_set_device")
    comm = Communicator.from_torch_distributed(transport="host")
    S = fd_laplacian_2d_sharded(-1.0, 1.0, M, comm)
    rng = np.random.default_rng(12345)
    rng.bit_generator.advance(S.row_begin)                            # x_exact rows of this rank
    b = psk.mvmult(S, rng.random(S.row_end - S.row_begin))            # halo exchange inside
    st = psk.PCG(control=_ctl(psk, 5), precond=psk.Jacobi()).makeSolver().solve(S, b)
    np.save(os.path.join(out_dir, "x%d.npy" % rank), st.soln())
    np.save(os.path.join(out_dir, "b%d.npy" % rank), b)
    np.savez(os.path.join(out_dir, "r%d.npz" % rank), hist=st.info["hist"], iters=st.iters(), ok=st.success(),
             rb=S.row_begin, re=S.row_end)
    del S
    dist.barrier()
    comm.destroy()
    dist.destroy_process_group()


def test_fd16384_sharded_p2_matches_unsharded(unsharded, tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    parts = [dict(np.load(tmp_path / ("r%d.npz" % r))) for r in range(world)]
    assert int(parts[0]["rb"]) == 0 and int(parts[-1]["re"]) == M * M
    assert int(parts[0]["re"]) == int(parts[1]["rb"]) and int(parts[0]["re"]) % M == 0   # whole grid lines
    b, hist, x = unsharded["b"], unsharded["hist5"], unsharded["x5"]
    for r, p in enumerate(parts):
        rb, re = int(p["rb"]), int(p["re"])
        assert np.array_equal(np.load(tmp_path / ("b%d.npy" % r)), b[rb:re])   # sharded SpMV bit-exact
        assert bool(p["ok"]) and int(p["iters"]) == unsharded["it5"] == 5
        assert np.array_equal(p["hist"], parts[0]["hist"])                   # identical scalars on every rank
        assert np.max(np.abs(p["hist"] - hist)) <= 1e-12 * np.linalg.norm(b)
        xr = np.load(tmp_path / ("x%d.npy" % r))
        assert np.linalg.norm(xr - x[rb:re]) <= 1e-12 * np.linalg.norm(x[rb:re])
