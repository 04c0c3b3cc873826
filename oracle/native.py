"""ORACLE — test infrastructure only (see oracle/__init__.py).

ctypes loader for the plain-C restatement in oracle/csr_matvec.c.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        lib.oracle_csr_matvec.argtypes = [ctypes.c_int64, P, P, P, P, P]
        lib.oracle_csr_diagonal.argtypes = [ctypes.c_int64, P, P, P, P]
        _lib = lib
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def csr_matvec(A, x):
    lib = _load()
    indptr = np.ascontiguousarray(A.indptr, dtype=np.int32)
    indices = np.ascontiguousarray(A.indices, dtype=np.int32)
    data = np.ascontiguousarray(A.data, dtype=np.float64)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty(A.shape[0], dtype=np.float64)
    lib.oracle_csr_matvec(A.shape[0], _ptr(indptr), _ptr(indices), _ptr(data), _ptr(x), _ptr(y))
    return y


def csr_diagonal(A):
    lib = _load()
    indptr = np.ascontiguousarray(A.indptr, dtype=np.int32)
    indices = np.ascontiguousarray(A.indices, dtype=np.int32)
    data = np.ascontiguousarray(A.data, dtype=np.float64)
    d = np.empty(A.shape[0], dtype=np.float64)
    lib.oracle_csr_diagonal(A.shape[0], _ptr(indptr), _ptr(indices), _ptr(data), _ptr(d))
    return d
