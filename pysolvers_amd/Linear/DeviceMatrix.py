"""HBM-resident operands: CSR matrices and f64 vectors owned by libpsk.

``DeviceCSR`` is what the solvers actually run on. ``LinearSolver.solve(A, b)``
(LinearSolver.py:30-33) accepts a scipy.sparse matrix exactly like the
reference and uploads it; passing a ``DeviceCSR`` (or freezing the matrix,
LinearSolver.freezeMatrix) keeps it resident across solves.
"""
import ctypes

import numpy as np
import scipy.sparse as sp

from .. import _native as N


class DeviceVector:
    """A length-n float64 vector in HBM (library-owned allocation)."""

    def __init__(self, n):
        self.n = int(n)
        p = ctypes.c_void_p()
        N.check(N.lib.psk_dmalloc(self.n * 8, ctypes.byref(p)), "psk_dmalloc")
        self._p = p

    @classmethod
    def from_numpy(cls, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        v = cls(a.shape[0])
        N.check(N.lib.psk_h2d(v._p, N.ptr(a), a.nbytes), "psk_h2d")
        return v

    def numpy(self):
        out = np.empty(self.n, dtype=np.float64)
        N.check(N.lib.psk_d2h(N.ptr(out), self._p, out.nbytes), "psk_d2h")
        return out

    def zero(self):
        N.check(N.lib.psk_dmemset0(self._p, self.n * 8), "psk_dmemset0")

    def data_ptr(self):
        return self._p.value or 0

    def __len__(self):
        return self.n

    @property
    def shape(self):
        return (self.n,)

    def __del__(self):
        try:
            if self._p:
                N.lib.psk_dfree(self._p)
                self._p = ctypes.c_void_p()
        except Exception:
            pass


def is_device_vector(v):
    """DeviceVector, or a contiguous float64 torch tensor on a GPU."""
    if isinstance(v, DeviceVector):
        return True
    return (hasattr(v, "is_cuda") and getattr(v, "is_cuda", False))


def torch_stream_ready(*tensors):
    """Order libpsk after torch for the torch tensors about to be handed to it.

    libpsk runs on its own non-blocking stream (runtime.hip), which nothing orders after torch's
    current stream: an input may still be written by a queued torch kernel, and an output fresh
    from the caching allocator may still be read by torch work on its previous use. So wait for
    torch's current stream on every device involved (allocate the outputs first). Every libpsk
    entry point synchronises its own stream before returning, so torch may use the results at
    once."""
    import torch
    for dev in {t.device for t in tensors if not isinstance(t, DeviceVector)}:
        torch.cuda.current_stream(dev).synchronize()


class DeviceCSR:
    """CSR matrix (int32 rowptr/colidx, float64 vals) in HBM; stored entry order is preserved."""

    def __init__(self, handle, n, nnz, comm=None, row_begin=0, row_end=None, n_global=None, ncols=None):
        self._h = handle
        self.n = int(n)
        self.ncols = int(n if ncols is None else ncols)
        self.nnz = int(nnz)
        self.comm = comm
        self.row_begin = int(row_begin)
        self.row_end = int(n if row_end is None else row_end)
        self.n_global = int(n if n_global is None else n_global)

    # --- constructors ---------------------------------------------------------------------
    @classmethod
    def from_scipy(cls, A, rectangular=False):
        """Upload a scipy matrix (CSR kept in its stored entry order). rectangular=True allows
        nrows != ncols (AMG transfer operators); solvers require square matrices."""
        if not sp.issparse(A):
            A = sp.csr_matrix(np.asarray(A, dtype=np.float64))
        A = A.tocsr()
        n, nc = A.shape
        if n != nc and not rectangular:
            raise AssertionError("matrix must be square")
        if A.nnz >= 2 ** 31:
            raise ValueError("int32 CSR required (nnz < 2^31)")
        indptr = np.ascontiguousarray(A.indptr, dtype=np.int32)
        indices = np.ascontiguousarray(A.indices, dtype=np.int32)
        data = np.ascontiguousarray(A.data, dtype=np.float64)
        h = ctypes.c_void_p()
        N.check(N.lib.psk_csr_create_rect(n, nc, A.nnz, N.ptr(indptr), N.ptr(indices), N.ptr(data), N.PSK_HOST,
                                          ctypes.byref(h)), "psk_csr_create_rect")
        return cls(h, n, A.nnz, ncols=nc)

    @classmethod
    def fd_laplacian_2d(cls, a, b, m):
        """FDLaplacian2D(a, b, m) built on the device (examples/FDLaplacian2D.py:5-23)."""
        h = ctypes.c_void_p()
        N.check(N.lib.psk_csr_create_fd2d(float(a), float(b), int(m), ctypes.byref(h)), "psk_csr_create_fd2d")
        n = int(m) * int(m)
        nnz = 1 if m == 1 else 5 * n - 4 * int(m)
        return cls(h, n, nnz)

    @classmethod
    def from_mtx(cls, path):
        """scipy.io.mmread(path).tocsr() read by the native MatrixMarket reader straight into HBM."""
        import os
        h = ctypes.c_void_p()
        N.check(N.lib.psk_csr_create_mm(os.fsencode(os.fspath(path)), ctypes.byref(h)), "psk_csr_create_mm")
        n, nnz = N.I64(), N.I64()
        N.check(N.lib.psk_csr_info(h, ctypes.byref(n), ctypes.byref(nnz)), "psk_csr_info")
        nr, nc, _ = __import__("pysolvers_amd.io", fromlist=["mm_info"]).mm_info(path)
        return cls(h, n.value, nnz.value, ncols=nc)

    # --- accessors ------------------------------------------------------------------------
    @property
    def shape(self):
        return (self.n, self.ncols) if self.comm is None else (self.n, self.n_global)

    @property
    def handle(self):
        return self._h

    _LAYOUTS = {"csr": 0, "sliced": 1, "sliced_wide": 2, "sliced_dict": 3, "diag": 4}

    @property
    def layout(self):
        """SpMV storage layout: "csr", "sliced" (16-bit column deltas where they fit), "sliced_wide"
        or "sliced_dict" (sliced + one-byte value indices into the matrix's <= 8 distinct values)
        (psk_csr_layout; y is bit-identical in every layout)."""
        k = N.I32()
        N.check(N.lib.psk_csr_layout(self._h, -1, ctypes.byref(k), None, None, None), "psk_csr_layout")
        return {v: n for n, v in self._LAYOUTS.items()}[k.value]

    def set_layout(self, layout):
        """Switch the SpMV storage layout; returns (padded slots, slots in 16-bit slices)."""
        slots, packed = N.I64(), N.I64()
        N.check(N.lib.psk_csr_layout(self._h, self._LAYOUTS[layout], None, ctypes.byref(slots), ctypes.byref(packed),
                                     None), "psk_csr_layout")
        return slots.value, packed.value

    def to_scipy(self):
        indptr = np.empty(self.n + 1, dtype=np.int32)
        indices = np.empty(self.nnz, dtype=np.int32)
        data = np.empty(self.nnz, dtype=np.float64)
        N.check(N.lib.psk_csr_download(self._h, N.ptr(indptr), N.ptr(indices), N.ptr(data)), "psk_csr_download")
        if self.comm is not None:
            return indptr, indices, data
        A = sp.csr_matrix((data, indices, indptr), shape=(self.n, self.ncols))
        A.has_sorted_indices = False
        return A

    def __del__(self):
        try:
            if self._h:
                N.lib.psk_csr_destroy(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


def as_device_matrix(A):
    if isinstance(A, DeviceCSR):
        return A
    return DeviceCSR.from_scipy(A)


def spmv(A, x):
    """y = A x on the device; bit-identical to scipy csr_matvec (stored-order row sums)."""
    dA = A if isinstance(A, DeviceCSR) else DeviceCSR.from_scipy(A, rectangular=True)
    if isinstance(x, DeviceVector):
        y = DeviceVector(dA.n)
        N.check(N.lib.psk_spmv(dA.handle, x._p, y._p, N.PSK_DEVICE), "psk_spmv")
        return y
    if is_device_vector(x):
        import torch
        y = torch.empty(dA.n, dtype=torch.float64, device=x.device)
        torch_stream_ready(x, y)
        N.check(N.lib.psk_spmv(dA.handle, N.ptr(x), N.ptr(y), N.PSK_DEVICE), "psk_spmv")
        return y
    x = np.ascontiguousarray(x, dtype=np.float64)
    if x.shape[0] != (dA.ncols if dA.comm is None else dA.n):
        raise ValueError("dimension mismatch")
    y = np.empty(dA.n, dtype=np.float64)
    N.check(N.lib.psk_spmv(dA.handle, N.ptr(x), N.ptr(y), N.PSK_HOST), "psk_spmv")
    return y
