"""The sharded PCG with P > 1 ranks on ONE GPU: P processes, each a rank on device 0, with the
collectives over the host shared-memory transport (psk_comm_init_host; RCCL refuses two ranks on one
device). Everything but the transport is the production multi-GPU path: shards, halo exchange of p
(contiguous and packed sends), allgathered dot products summed in rank order, host poll schedule.
The gathered solution must match the serial oracle (identical iteration count, residual history
within 1e-10 of ||b||, solution within 1e-10), and every rank must report bit-identical histories."""
import os
import socket

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _matrix(name):
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import golden_matrix, load_golden
    from oracle import fdlap
    if name.startswith("fd"):
        return fdlap.fd_laplacian_2d(-1.0, 1.0, int(name[2:]))
    return golden_matrix(load_golden("pcg_%s_identity.npz" % name))


def _worker(rank, world, port, name, kind, out_dir, mailbox=False):
    import sys
    sys.path.insert(0, REPO)
    import torch.distributed as dist
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    from pysolvers_amd.Linear.Distributed import Communicator, fd_laplacian_2d_sharded, shard_csr
    from oracle import fdlap
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    N.check(N.lib.psk_set_device(0), "psk_set_device")
    comm = Communicator.from_torch_distributed(transport="host", mailbox=mailbox)
    if mailbox:
        comm.check_mailbox(4)   # psk_comm_mailbox_check: known values through the exchange first
    A = _matrix(name)
    b, _ = fdlap.manufactured_rhs(A, 12345)
    if kind == "fd":
        S = fd_laplacian_2d_sharded(-1.0, 1.0, int(name[2:]), comm)
    else:
        S = shard_csr(A, comm)
    ctl = psk.CommonSolverArgs(maxiter=4000, tau=1e-8, showIters=False, showFinal=False)
    st = psk.PCG(control=ctl, precond=psk.Jacobi()).makeSolver().solve(S, b[S.row_begin:S.row_end])
    np.savez(os.path.join(out_dir, "r%d.npz" % rank), x=st.soln(), hist=st.info["hist"], iters=st.iters(),
             ok=st.success(), rb=S.row_begin, re=S.row_end)
    del S
    dist.barrier()
    comm.destroy()
    dist.destroy_process_group()


# fd512 x 2: shards of 128 slices whose first/last slices (halo lines) keep 32-bit columns while the
# rest are packed — the sliced SpMV layout across the halo
# overlap: PSK_HALO_OVERLAP=1, the halo exchange on a second stream overlapping K3 (opt-in)
# mailbox: the ranks' dot products through the host-shared mailbox (psk_comm_mailbox: kernel stores +
# one-wave gather kernels) instead of the transport's all-gathers; must give the same bits
@pytest.mark.parametrize("name,kind,world,overlap,mailbox", [
    ("fd64", "fd", 2, 0, 0), ("fd96", "fd", 3, 0, 0), ("dh12", "general", 3, 0, 0), ("fd50", "general", 4, 0, 0),
    ("fd512", "fd", 2, 0, 0), ("fd512", "fd", 2, 1, 0), ("fd96", "fd", 3, 1, 0),
    ("fd64", "fd", 2, 0, 1), ("fd96", "fd", 3, 1, 1), ("dh12", "general", 3, 0, 1), ("fd50", "general", 4, 0, 1),
    ("fd512", "fd", 4, 1, 1)])
def test_multirank_pcg_on_one_gpu(tmp_path, monkeypatch, name, kind, world, overlap, mailbox):
    import torch.multiprocessing as mp
    from oracle import fdlap, krylov
    monkeypatch.setenv("PSK_HALO_OVERLAP", str(overlap))   # inherited by the spawned ranks
    mp.start_processes(_worker, args=(world, _free_port(), name, kind, str(tmp_path), bool(mailbox)), nprocs=world,
                       join=True, start_method="spawn")
    parts = [dict(np.load(tmp_path / ("r%d.npz" % r))) for r in range(world)]
    A = _matrix(name)
    b, _ = fdlap.manufactured_rhs(A, 12345)
    ref = krylov.pcg(A, b, maxiter=4000, tau=1e-8, precond=krylov.jacobi_form(A))
    assert [int(p["rb"]) for p in parts][0] == 0 and int(parts[-1]["re"]) == A.shape[0]
    x = np.concatenate([p["x"] for p in parts])
    for p in parts:
        assert bool(p["ok"]) and int(p["iters"]) == ref["iters"]
        assert np.array_equal(p["hist"], parts[0]["hist"])            # identical scalars on every rank
        assert np.max(np.abs(p["hist"] - ref["hist"])) <= 1e-10 * np.linalg.norm(b)
    assert np.linalg.norm(x - ref["soln"]) <= 1e-10 * np.linalg.norm(ref["soln"])
