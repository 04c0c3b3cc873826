"""Abstract solver factory and solver (LinearSolver.py:7-42)."""
from abc import ABC, abstractmethod

from ..IterativeSolver import NamedObject


class LinearSolverType(ABC, NamedObject):
    def __init__(self, name=''):
        NamedObject.__init__(self, name=name)

    @abstractmethod
    def makeSolver(self, name=None):
        ...


class LinearSolver(ABC, NamedObject):
    """solve(A, b) -> SolveStatus; freezeMatrix() lets the device copy of A be reused."""

    def __init__(self, name=''):
        NamedObject.__init__(self, name=name)
        self._matrixFrozen = False

    @abstractmethod
    def solve(self, A, b):
        ...

    def freezeMatrix(self):
        self._matrixFrozen = True

    def unfreezeMatrix(self):
        self._matrixFrozen = False

    def matrixFrozen(self):
        return self._matrixFrozen
