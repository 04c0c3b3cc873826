"""MatrixMarket input through the native reader (pysolvers_amd/csrc/mmio.hip).

``mmread_csr(path)`` == ``scipy.io.mmread(path).tocsr()`` (examples/DHTestProblem.py:27-28) for
coordinate files, as a float64 CSR; ``DeviceCSR.from_mtx`` reads straight into HBM.
"""
import ctypes
import os

import numpy as np
import scipy.sparse as sp

from . import _native as N


def _path(p):
    return os.fsencode(os.fspath(p))


def mm_info(path):
    r, c, z = N.I64(), N.I64(), N.I64()
    N.check(N.lib.psk_mm_info(_path(path), ctypes.byref(r), ctypes.byref(c), ctypes.byref(z)), "psk_mm_info")
    return r.value, c.value, z.value


def mmread_csr(path):
    nr, nc, zmax = mm_info(path)
    rp = np.empty(nr + 1, dtype=np.int32)
    ci = np.empty(max(zmax, 1), dtype=np.int32)
    va = np.empty(max(zmax, 1), dtype=np.float64)
    nnz = N.I64()
    N.check(N.lib.psk_mm_read(_path(path), N.ptr(rp), N.ptr(ci), N.ptr(va), ctypes.byref(nnz)), "psk_mm_read")
    k = nnz.value
    return sp.csr_matrix((va[:k].copy(), ci[:k].copy(), rp), shape=(nr, nc))
