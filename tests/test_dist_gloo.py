"""N>1 path on CPU: world_size 2 and 3 over gloo.

The product's sharding plan (psk_fd2d_dist_plan, the exact function psk_csr_create_fd2d_dist
uses) drives a row-block distributed PCG restatement (oracle/dist_pcg.py) with the engine's
communication schedule (halo exchange with r+-1, sum-all-reduce of dot partials). The gathered
result must match the serial oracle: identical iteration count, residual history within 1e-10 of
||b||.
"""
import os
import socket

import numpy as np
import pytest

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, m, out_dir):
    import sys
    sys.path.insert(0, REPO)
    import torch.distributed as dist
    from oracle import dist_pcg, fdlap
    from pysolvers_amd import _native as N
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    plan = N.fd2d_dist_plan(m, world, rank)
    rb, re = plan[0], plan[1]
    Aloc = dist_pcg.local_block(m, plan)
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    b, _ = fdlap.manufactured_rhs(A, 12345)
    st = dist_pcg.dist_pcg(dist, m, Aloc, b[rb:re], plan, maxiter=4000, tau=1e-8)
    np.savez(os.path.join(out_dir, "r%d.npz" % rank), x=st["x"], hist=st["hist"], iters=st["iters"],
             rb=rb, re=re)
    dist.barrier()
    dist.destroy_process_group()


def test_plan_covers_rows_once():
    from pysolvers_amd import _native as N
    for m in (1, 2, 7, 64, 1000):
        for P in range(1, min(m, 9) + 1):
            prev = 0
            for r in range(P):
                rb, re, ncols, hlo, hhi = N.fd2d_dist_plan(m, P, r)
                assert rb == prev and rb % m == 0 and re % m == 0 and re > rb
                assert hlo == (m if r > 0 else 0) and hhi == (m if r < P - 1 else 0)
                assert ncols == re - rb + hlo + hhi
                prev = re
            assert prev == m * m


def test_plan_rejects_too_many_ranks():
    from pysolvers_amd import _native as N
    with pytest.raises(N.PskError):
        N.fd2d_dist_plan(4, 5, 0)


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_pcg_matches_serial(tmp_path, world):
    import torch.multiprocessing as mp
    from oracle import fdlap, krylov
    m = 64
    mp.start_processes(_worker, args=(world, _free_port(), m, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    parts = [dict(np.load(tmp_path / ("r%d.npz" % r))) for r in range(world)]
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    b, _ = fdlap.manufactured_rhs(A, 12345)
    ref = krylov.pcg(A, b, maxiter=4000, tau=1e-8, precond=krylov.jacobi_form(A))
    x = np.concatenate([p["x"] for p in parts])
    for p in parts:
        assert int(p["iters"]) == ref["iters"] == 177
        assert np.max(np.abs(p["hist"] - ref["hist"])) <= 1e-10 * np.linalg.norm(b)
    assert np.linalg.norm(x - ref["soln"]) <= 1e-10 * np.linalg.norm(ref["soln"])


# ---- general row-block sharding (psk_csr_create_dist / pysolvers_amd.Linear.shard_csr) ---------
def _general_matrix(name):
    from conftest import golden_matrix, load_golden
    from oracle import fdlap
    if name == "fd40":
        return fdlap.fd_laplacian_2d(-1.0, 1.0, 40)
    return golden_matrix(load_golden("pcg_%s_identity.npz" % name))


@pytest.mark.parametrize("name", ["dh8", "dh12", "fd40"])
@pytest.mark.parametrize("world", [2, 3, 5])
def test_general_plan_send_lists_are_peer_receives(name, world):
    """The symmetric-pattern premise psk_csr_create_dist builds its send lists on: what rank r sends
    q (owned rows with an entry in q's block) is exactly q's received halo segment from r."""
    from pysolvers_amd.Linear.Distributed import even_row_starts
    from oracle import dist_pcg
    A = _general_matrix(name)
    rs = even_row_starts(A.shape[0], world, A.indptr)
    assert rs[0] == 0 and rs[-1] == A.shape[0] and np.all(np.diff(rs) >= 0)
    plans = [dist_pcg.shard_plan(A, rs, r) for r in range(world)]
    for r, pr in enumerate(plans):
        assert set(pr["send"]) == set(pr["recv"])
        for q, rows in pr["send"].items():
            off, cnt = plans[q]["recv"][r]
            assert np.array_equal(plans[q]["halo"][off:off + cnt], pr["rb"] + rows)
        # the local block reproduces the global rows: same stored order, columns remapped
        xg = np.random.default_rng(r).standard_normal(A.shape[0])
        xe = np.concatenate([xg[pr["rb"]:pr["re"]], xg[pr["halo"]]])
        assert np.array_equal(pr["Aloc"] @ xe, (A @ xg)[pr["rb"]:pr["re"]])


def _general_worker(rank, world, port, name, out_dir):
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch.distributed as dist
    from oracle import dist_pcg, fdlap
    from pysolvers_amd.Linear.Distributed import even_row_starts
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    A = _general_matrix(name)
    b, _ = fdlap.manufactured_rhs(A, 12345)
    rs = even_row_starts(A.shape[0], world, A.indptr)
    plan = dist_pcg.shard_plan(A, rs, rank)
    st = dist_pcg.dist_pcg_general(dist, plan, b[plan["rb"]:plan["re"]], maxiter=4000, tau=1e-8)
    np.savez(os.path.join(out_dir, "g%d.npz" % rank), x=st["x"], hist=st["hist"], iters=st["iters"])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("dh12", 2), ("dh12", 3), ("fd40", 3)])
def test_general_distributed_pcg_matches_serial(tmp_path, name, world):
    import torch.multiprocessing as mp
    from oracle import fdlap, krylov
    mp.start_processes(_general_worker, args=(world, _free_port(), name, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    parts = [dict(np.load(tmp_path / ("g%d.npz" % r))) for r in range(world)]
    A = _general_matrix(name)
    b, _ = fdlap.manufactured_rhs(A, 12345)
    ref = krylov.pcg(A, b, maxiter=4000, tau=1e-8, precond=krylov.jacobi_form(A))
    x = np.concatenate([p["x"] for p in parts])
    for p in parts:
        assert int(p["iters"]) == ref["iters"]
        assert np.max(np.abs(p["hist"] - ref["hist"])) <= 1e-10 * np.linalg.norm(b)
    assert np.linalg.norm(x - ref["soln"]) <= 1e-10 * np.linalg.norm(ref["soln"])
