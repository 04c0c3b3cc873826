"""ORACLE — test infrastructure only (see oracle/__init__.py).

Vectorised restatement of the reference's problem generators.

``fd_laplacian_2d`` reproduces ``examples/FDLaplacian2D.py:5-23`` bit for bit,
including the CSR entry order that ``dok_matrix.tocsr()`` leaves behind.  The
reference inserts, for grid point k = m*iy + ix, the keys (k,k), (k,k-m),
(k,k+m), (k,k-1), (k,k+1) in that order (FDLaplacian2D.py:13-21); the DOK ->
COO -> CSR conversion is stable per row, so every CSR row is stored as
[diag, -m, +m, -1, +1] with boundary neighbours omitted (indices NOT sorted).
Values are ``-4.0/h/h`` and ``1.0/h/h`` with ``h = abs(b-a)/double(m+1)``
(FDLaplacian2D.py:6,13,15).
"""
import numpy as np
import scipy.sparse as sp


def fd_laplacian_2d_arrays(a, b, m):
    """Return (indptr int32, indices int32, data float64) of FDLaplacian2D(a,b,m)."""
    m = int(m)
    n = m * m
    h = np.abs(b - a) / np.double(m + 1)          # FDLaplacian2D.py:6
    diag = -4.0 / h / h                           # :13
    off = 1.0 / h / h                             # :15-21
    it = np.int32 if 5 * n < 2 ** 31 else np.int64
    k = np.arange(n, dtype=it)
    ix = k % m
    iy = k // m
    # slot order per row: diag, -m, +m, -1, +1  (insertion order, :13-21); filled slot by slot
    # so that peak memory stays a few vectors (m = 16384 has 1.34e9 entries)
    slots = [(None, None), (iy > 0, -m), (iy < m - 1, m), (ix > 0, -1), (ix < m - 1, 1)]
    counts = np.ones(n, dtype=np.int8)
    for mask, _ in slots[1:]:
        counts += mask
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    del counts
    nnz = int(indptr[-1])
    indices = np.empty(nnz, dtype=np.int32)
    data = np.empty(nnz, dtype=np.float64)
    pos = indptr[:-1].copy()
    indices[pos] = k
    data[pos] = diag
    pos += 1
    for mask, d in slots[1:]:
        p = pos[mask]
        indices[p] = k[mask] + d
        data[p] = off
        pos[mask] += 1
        del p
    return indptr.astype(np.int32), indices, data


def fd_laplacian_2d(a, b, m):
    """scipy CSR identical (arrays and entry order) to examples/FDLaplacian2D.py."""
    indptr, indices, data = fd_laplacian_2d_arrays(a, b, m)
    n = int(m) * int(m)
    A = sp.csr_matrix((data, indices, indptr), shape=(n, n))
    A.has_sorted_indices = False
    return A


def fd_rowptr_closed_form(m, k):
    """Closed-form rowptr[k] of the m x m 5-point stencil (used by the device generator).

    rowptr[k] = 5k - #(iy==0) - #(iy==m-1) - #(ix==0) - #(ix==m-1) over rows < k.
    """
    k = np.asarray(k, dtype=np.int64)
    return (5 * k - np.minimum(k, m) - np.maximum(0, k - m * (m - 1))
            - (k + m - 1) // m - k // m)


def manufactured_rhs(A, seed=12345):
    """x_exact = default_rng(seed).random(n), b = A @ x_exact (DHTestProblem.py:53-57, seeded)."""
    n = A.shape[0]
    x = np.random.default_rng(seed).random(n)
    b = A @ x
    return b, x


class FDStencil:
    """FDLaplacian2D(a, b, m) as a matrix-free operator whose ``@`` is bit-identical to scipy
    csr_matvec on the CSR that ``fd_laplacian_2d`` (= the reference generator) builds: every row is
    summed from 0.0 in stored order [diag, -m, +m, -1, +1] with rounded products, absent neighbours
    skipped (IterativeLinearSolver.py:104 -> csr_matvec; FDLaplacian2D.py:13-21). Vectorised over
    rows in that slot order, so configs[3]'s m = 16384 (1.34e9 entries) needs no 16 GB CSR on the
    host: only a few n-vectors. Has what oracle/krylov.py reads from a matrix: shape, diagonal(),
    ``@``. tests/test_oracle_golden.py pins it to the CSR product."""

    def __init__(self, a, b, m):
        self.m = int(m)
        n = self.m * self.m
        self.shape = (n, n)
        h = np.abs(b - a) / np.double(m + 1)          # FDLaplacian2D.py:6
        self.dval = -4.0 / h / h                      # :13
        self.oval = 1.0 / h / h                       # :15-21

    def diagonal(self):
        return np.full(self.shape[0], self.dval)

    def __matmul__(self, x):
        m = self.m
        x = np.asarray(x, dtype=np.float64)
        y = np.add(0.0, self.dval * x)                # sum = 0; sum += diag * x_k (0.0 + -0.0 = +0.0 as in C)
        if m > 1:
            y[m:] += self.oval * x[:-m]               # -m neighbour: rows with iy > 0
            y[:-m] += self.oval * x[m:]               # +m: iy < m-1
            Y, X = y.reshape(m, m), x.reshape(m, m)
            Y[:, 1:] += self.oval * X[:, :-1]         # -1: ix > 0
            Y[:, :-1] += self.oval * X[:, 1:]         # +1: ix < m-1
        return y
