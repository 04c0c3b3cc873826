"""ILUT preconditioners (ILUTPreconditioner.py:1-78): factors on the host, apply on the GPU.

``form(A)`` makes exactly the reference's SuperLU call,
``spilu(A.tocsc(), drop_tol, fill_factor, diag_pivot_thresh=0.0)`` (ILUTPreconditioner.py:51-53)
— the factorisation is setup, done once per form() by the same third-party library — then
uploads L, U, perm_r, perm_c once (``psk_prec_create_ilu``). ``applyRight`` (the operator
PCG/GMRES call inside the loop, :77-78) runs the two sparse triangular solves on the device.
As in the reference, a LEFT ILUT is the identity when applied from the right
(Preconditioner.py:39-46), so right-preconditioned solvers ignore it.
"""
import ctypes

import numpy as np
import scipy.sparse.linalg as spla

from .. import _native as N
from .DeviceMatrix import DeviceCSR
from .Preconditioner import DeviceOperator, LeftPreconditioner, Preconditioner, RightPreconditioner
from .PreconditionerType import PreconditionerType


def _host_matrix(A):
    return A.to_scipy() if isinstance(A, DeviceCSR) else A


class LeftILUT(PreconditionerType):
    def __init__(self, drop_tol=0.001, fill_factor=15):
        self.drop_tol = drop_tol
        self.fill_factor = fill_factor

    def form(self, A):
        return LeftILUTPreconditioner(A, drop_tol=self.drop_tol, fill_factor=self.fill_factor)


class RightILUT(PreconditionerType):
    def __init__(self, drop_tol=0.001, fill_factor=15):
        self.drop_tol = drop_tol
        self.fill_factor = fill_factor

    def form(self, A):
        return RightILUTPreconditioner(A, drop_tol=self.drop_tol, fill_factor=self.fill_factor)


class ILUTPreconditioner(DeviceOperator, Preconditioner):
    def __init__(self, A, drop_tol=0.001, fill_factor=15):
        Ah = _host_matrix(A)
        self._ILU = spla.spilu(Ah.tocsc(), drop_tol=drop_tol, fill_factor=fill_factor, diag_pivot_thresh=0.0)
        L = self._ILU.L.tocsr()
        U = self._ILU.U.tocsr()
        self.n = Ah.shape[0]
        arr = [np.ascontiguousarray(a, dtype=t) for a, t in (
            (L.indptr, np.int32), (L.indices, np.int32), (L.data, np.float64),
            (U.indptr, np.int32), (U.indices, np.int32), (U.data, np.float64),
            (self._ILU.perm_r, np.int32), (self._ILU.perm_c, np.int32))]
        h = ctypes.c_void_p()
        N.check(N.lib.psk_prec_create_ilu(self.n, *[N.ptr(a) for a in arr], ctypes.byref(h)), "psk_prec_create_ilu")
        self._h = h

    def ILU(self):
        return self._ILU


class LeftILUTPreconditioner(ILUTPreconditioner, LeftPreconditioner):
    """applyRight is the identity (Preconditioner.py:44-45)."""

    device_kind = N.PSK_PREC_IDENTITY
    device_handle = None

    def applyLeft(self, vec):
        return self._device_apply(vec)


class RightILUTPreconditioner(ILUTPreconditioner, RightPreconditioner):
    device_kind = N.PSK_PREC_ILU

    def applyRight(self, vec):
        return self._device_apply(vec)
