"""Row-block sharding across the GPUs of one node (one process per GPU, RCCL over xGMI).

The reference is single-process; this is the multi-GPU path of the north star.
A sharded ``DeviceCSR`` holds one rank's rows with local columns ``[owned | halo]``; handing it to
the unchanged solver API (``PCG(...).makeSolver().solve(A_shard, b_local)``) runs the sharded PCG
(halo exchange of p with ncclSend/ncclRecv, rank-ordered sums of allgathered dot products), and
``SolveStatus.soln()`` is this rank's block of x. Every rank takes identical branches and stops on
the same iteration.

    comm = Communicator.from_torch_distributed()          # torch.distributed already initialised
    A_r = shard_csr(A, comm)                             # or DeviceCSR.fd_laplacian_2d_sharded
    st = PCG(control=ctl, precond=Jacobi()).makeSolver().solve(A_r, b[A_r.row_begin:A_r.row_end])
"""
import ctypes

import numpy as np
import scipy.sparse as sp

from .. import _native as N
from .DeviceMatrix import DeviceCSR


class Communicator:
    """A psk_comm: RCCL communicator of `nranks` (production), a dry one (shards without
    collectives) or a host shared-memory one (transport="host": the collectives of P processes on
    ONE GPU, for validating the multi-rank path where RCCL refuses duplicate devices)."""

    def __init__(self, nranks, rank, unique_id=None, dry=False, transport="rccl"):
        self.nranks, self.rank, self.dry = int(nranks), int(rank), bool(dry)
        self.transport = "dry" if dry else transport
        h = ctypes.c_void_p()
        if dry:
            N.check(N.lib.psk_comm_init_dry(self.nranks, self.rank, ctypes.byref(h)), "psk_comm_init_dry")
        elif transport == "host":
            if not unique_id:
                raise ValueError("Communicator(transport='host'): unique_id = shared segment name '/...'")
            name = unique_id if isinstance(unique_id, bytes) else str(unique_id).encode()
            N.check(N.lib.psk_comm_init_host(self.nranks, self.rank, name, ctypes.byref(h)), "psk_comm_init_host")
        elif transport != "rccl":
            raise ValueError("transport must be 'rccl' or 'host'")
        else:
            if unique_id is None:
                raise ValueError("Communicator: unique_id required (Communicator.unique_id() on rank 0)")
            uid = (ctypes.c_uint8 * N.PSK_UNIQUE_ID_BYTES).from_buffer_copy(bytes(unique_id))
            N.check(N.lib.psk_comm_init(self.nranks, self.rank, uid, ctypes.byref(h)), "psk_comm_init")
        self._h = h
        self.mailbox = None

    @staticmethod
    def unique_id():
        uid = (ctypes.c_uint8 * N.PSK_UNIQUE_ID_BYTES)()
        N.check(N.lib.psk_comm_unique_id(uid), "psk_comm_unique_id")
        return bytes(uid)

    @classmethod
    def from_torch_distributed(cls, group=None, transport="rccl", mailbox=False):
        """Collective over the torch.distributed group (any backend; gloo is enough, it only
        carries the RCCL unique id / the shared segment names). mailbox=True also attaches the
        host-shared mailbox of the device-side scalar exchange (attach_mailbox; ranks on one node)."""
        import os
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = mbn = None
        if rank == 0:
            uid = cls.unique_id() if transport == "rccl" else ("/psk_%d_%s" % (os.getpid(), os.urandom(6).hex())).encode()
            mbn = ("/psk_mb_%d_%s" % (os.getpid(), os.urandom(6).hex())).encode()
        obj = [uid, mbn]
        dist.broadcast_object_list(obj, src=0, group=group)
        comm = cls(world, rank, obj[0], transport=transport)
        if mailbox:
            comm.attach_mailbox(obj[1])
        return comm

    def attach_mailbox(self, name):
        """psk_comm_mailbox (collective, one node): the sharded PCG then exchanges its per-rank dot
        products through kernel stores into a host-shared mailbox instead of all-gathers; same bits."""
        name = name if isinstance(name, bytes) else str(name).encode()
        N.check(N.lib.psk_comm_mailbox(self._h, name), "psk_comm_mailbox")
        self.mailbox = name

    def check_mailbox(self, rounds=4):
        """psk_comm_mailbox_check (collective): known values through the mailbox exchange; raises on a wrong
        or missing value (bounded waits)."""
        N.check(N.lib.psk_comm_mailbox_check(self._h, int(rounds)), "psk_comm_mailbox_check")

    @property
    def handle(self):
        return self._h

    def destroy(self):
        if self._h:
            N.lib.psk_comm_destroy(self._h)
            self._h = ctypes.c_void_p()


def even_row_starts(n, nranks, indptr=None):
    """Row split of n rows over nranks: balanced by stored entries when indptr is given (the SpMV
    stream dominates the iteration), else by rows. Returns int64[nranks+1]."""
    if indptr is None:
        return np.array([n * q // nranks for q in range(nranks + 1)], dtype=np.int64)
    nnz = int(indptr[-1])
    rs = np.searchsorted(np.asarray(indptr, dtype=np.int64), [nnz * q // nranks for q in range(nranks + 1)])
    rs = np.asarray(rs, dtype=np.int64)
    rs[0], rs[-1] = 0, n
    return np.maximum.accumulate(rs)


def shard_csr(A, comm, row_starts=None):
    """This rank's row block of the global scipy matrix A (stored entry order kept) as a sharded
    DeviceCSR. The pattern must be structurally symmetric (psk_csr_create_dist)."""
    A = A.tocsr() if sp.issparse(A) else sp.csr_matrix(np.asarray(A, dtype=np.float64))
    n, nc = A.shape
    if n != nc:
        raise AssertionError("matrix must be square")
    if row_starts is None:
        row_starts = even_row_starts(n, comm.nranks, A.indptr)
    rs = np.ascontiguousarray(row_starts, dtype=np.int64)
    if rs.shape[0] != comm.nranks + 1:
        raise ValueError("row_starts must hold nranks+1 entries")
    rb, re = int(rs[comm.rank]), int(rs[comm.rank + 1])
    rp = np.ascontiguousarray(A.indptr[rb:re + 1], dtype=np.int64)
    e0, e1 = int(rp[0]), int(rp[-1])
    ci = np.ascontiguousarray(A.indices[e0:e1], dtype=np.int32)
    dt = np.ascontiguousarray(A.data[e0:e1], dtype=np.float64)
    h = ctypes.c_void_p()
    N.check(N.lib.psk_csr_create_dist(n, N.ptr(rs), N.ptr(rp), N.ptr(ci), N.ptr(dt), comm.handle, ctypes.byref(h)),
            "psk_csr_create_dist")
    nh = N.I64()
    N.check(N.lib.psk_csr_halo_cols(h, None, ctypes.byref(nh)), "psk_csr_halo_cols")
    return DeviceCSR(h, re - rb, e1 - e0, comm=comm, row_begin=rb, row_end=re, n_global=n,
                     ncols=re - rb + nh.value)


def fd_laplacian_2d_sharded(a, b, m, comm):
    """Rank comm.rank's whole-grid-line block of FDLaplacian2D(a, b, m), built on the device."""
    h = ctypes.c_void_p()
    rb, re = N.I64(), N.I64()
    N.check(N.lib.psk_csr_create_fd2d_dist(float(a), float(b), int(m), comm.handle, ctypes.byref(h),
                                           ctypes.byref(rb), ctypes.byref(re)), "psk_csr_create_fd2d_dist")
    nnz, nh = N.I64(), N.I64()
    N.check(N.lib.psk_csr_info(h, None, ctypes.byref(nnz)), "psk_csr_info")
    N.check(N.lib.psk_csr_halo_cols(h, None, ctypes.byref(nh)), "psk_csr_halo_cols")
    return DeviceCSR(h, re.value - rb.value, nnz.value, comm=comm, row_begin=rb.value, row_end=re.value,
                     n_global=int(m) * int(m), ncols=re.value - rb.value + nh.value)


def halo_cols(A):
    """Global index of each halo column of a sharded DeviceCSR (local column order)."""
    nh = N.I64()
    N.check(N.lib.psk_csr_halo_cols(A.handle, None, ctypes.byref(nh)), "psk_csr_halo_cols")
    out = np.empty(nh.value, dtype=np.int64)
    N.check(N.lib.psk_csr_halo_cols(A.handle, N.ptr(out), ctypes.byref(nh)), "psk_csr_halo_cols")
    return out
