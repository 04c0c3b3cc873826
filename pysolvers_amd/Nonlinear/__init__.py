"""Nonlinear callers of the device Krylov solvers (PySolvers/Nonlinear: Newton.py, LineSearch.py,
PreconditionerFreeze.py). The Newton loop, the function evaluations and the line search stay on the
host, as in the reference; every Newton step's linear solve is the device PCG/GMRES."""
from .LineSearch import LineSearch, SimpleBacktrack, TrivialLinesearch
from .Newton import NewtonSolver
from .PreconditionerFreeze import PreconditionerFreeze
