"""Preconditioner plugin classes (same hierarchy as Linear/Preconditioner.py:3-68).

Preconditioners that run inside the device Krylov loop expose a ``device_kind``
and a ``device_handle`` (a libpsk psk_prec*). ``applyLeft/applyRight`` keep the
reference's host-callable contract: they take and return a vector.
"""
import ctypes
from abc import ABC, abstractmethod

import numpy as np

from .. import _native as N
from .DeviceMatrix import DeviceVector, as_device_matrix, is_device_vector, torch_stream_ready


class Preconditioner(ABC):
    """Two-sided preconditioner interface (Preconditioner.py:3-18)."""

    device_kind = None

    @abstractmethod
    def applyLeft(self, vec):
        ...

    @abstractmethod
    def applyRight(self, vec):
        ...


class GenericPreconditioner(Preconditioner):
    """Same operator on either side (Preconditioner.py:20-36)."""

    @abstractmethod
    def apply(self, vec):
        ...

    def applyLeft(self, vec):
        return self.apply(vec)

    def applyRight(self, vec):
        return self.apply(vec)


class LeftPreconditioner(Preconditioner):
    """applyRight is the identity (Preconditioner.py:39-46)."""

    def applyRight(self, vec):
        return vec


class RightPreconditioner(Preconditioner):
    """applyLeft is the identity (Preconditioner.py:49-56)."""

    def applyLeft(self, vec):
        return vec


class IdentityPreconditioner:
    """Returns its argument itself (Preconditioner.py:58-68); duck-typed like the reference."""

    device_kind = N.PSK_PREC_IDENTITY
    device_handle = None

    def applyLeft(self, vec):
        return vec

    def applyRight(self, vec):
        return vec


class DeviceOperator:
    """Mixin for preconditioners backed by a libpsk psk_prec handle (self._h, size self.n).

    ``_device_apply`` takes a DeviceVector, a CUDA float64 tensor or a host array and returns the
    same kind; the operator itself always runs on the GPU.
    """

    _h = None
    device_kind = None

    @property
    def device_handle(self):
        return self._h

    def _device_apply(self, vec):
        if isinstance(vec, DeviceVector):
            out = DeviceVector(self.n)
            N.check(N.lib.psk_prec_apply(self._h, self.n, vec._p, out._p, N.PSK_DEVICE), "psk_prec_apply")
            return out
        if is_device_vector(vec):
            import torch
            out = torch.empty_like(vec)
            torch_stream_ready(vec, out)
            N.check(N.lib.psk_prec_apply(self._h, self.n, N.ptr(vec), N.ptr(out), N.PSK_DEVICE), "psk_prec_apply")
            return out
        v = np.ascontiguousarray(vec, dtype=np.float64)
        out = np.empty_like(v)
        N.check(N.lib.psk_prec_apply(self._h, self.n, N.ptr(v), N.ptr(out), N.PSK_HOST), "psk_prec_apply")
        return out

    def device_info(self):
        """kind / size / triangular-solve nnz and dependency levels (psk_prec_info)."""
        return N.prec_info(self._h)

    def __del__(self):
        try:
            if self._h:
                N.lib.psk_prec_destroy(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


class JacobiPreconditioner(DeviceOperator, GenericPreconditioner):
    """M^-1 v = DInv * v with DInv = reciprocal(diag(A)) formed on the device.

    The reference has Jacobi only as a smoother (ClassicSmoothers.py:5-16:
    ``DInv = np.reciprocal(A.diagonal())``; ``np.multiply(DInv, r)``); this is
    the same operator behind the PreconditionerType plugin API, as config 2 of
    the benchmark needs (PCG + Jacobi).
    """

    device_kind = N.PSK_PREC_JACOBI

    def __init__(self, A):
        self._A = as_device_matrix(A)        # keep the matrix alive as long as DInv
        h = ctypes.c_void_p()
        N.check(N.lib.psk_prec_create(self._A.handle, N.PSK_PREC_JACOBI, ctypes.byref(h)), "psk_prec_create")
        self._h = h
        self.n = self._A.n

    def apply(self, vec):
        return self._device_apply(vec)
