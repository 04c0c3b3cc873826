"""Preconditioner factories (PreconditionerType.py:4-19): ``form(A)`` builds the operator."""
from abc import ABC, abstractmethod

from .Preconditioner import IdentityPreconditioner, JacobiPreconditioner


class PreconditionerType(ABC):
    @abstractmethod
    def form(self, A):
        ...


class IdentityPreconditionerType(PreconditionerType):
    """PreconditionerType.py:13-19."""

    def form(self, A):
        return IdentityPreconditioner()


class JacobiPreconditionerType(PreconditionerType):
    """Point-Jacobi (DInv = 1/diag(A)), the preconditioner of benchmark config 2."""

    def form(self, A):
        return JacobiPreconditioner(A)


# short factory name in the style of RightILUT()/RightIC()/AMG()
Jacobi = JacobiPreconditionerType
