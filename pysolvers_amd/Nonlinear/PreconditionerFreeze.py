"""Freeze the linear solver's preconditioner across Newton steps (PreconditionerFreeze.py:3-24)."""
from ..Linear.IterativeLinearSolver import IterativeLinearSolver


class PreconditionerFreeze:
    """Freezes on construction; ``unfreeze()`` releases. (The reference names its releasing hook
    ``__def__`` (:23), so it never runs automatically and the solver stays frozen after the solve;
    the same happens here.)"""

    def __init__(self, solver, freezePrec):
        self.solver = solver
        self.freezePrec = freezePrec
        self.freeze()

    def freeze(self):
        if self.freezePrec and isinstance(self.solver, IterativeLinearSolver):
            self.solver.freezePrec()

    def unfreeze(self):
        if self.freezePrec and isinstance(self.solver, IterativeLinearSolver):
            self.solver.unfreezePrec()
