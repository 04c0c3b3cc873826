"""pysolvers_amd — MI355X-native Krylov engine behind the PySolvers.Linear solver API.

Importing this package loads libpsk.so (hand-written gfx950 HIP kernels);
there is no CPU fallback.
"""
from . import Linear, Nonlinear, io
from .IterativeSolver import CommonSolverArgs, IterativeSolver, NamedObject, SolveStatus
from .Linear import (AMG, DefaultDirect, GMRES, PCG, RightIC, GaussSeidelSmoother, JacobiSmoother, DeviceCSR, DeviceVector, GMRESSolver, IdentityPreconditioner,
                     IdentityPreconditionerType, IterativeLinearSolver, Jacobi, JacobiPreconditioner,
                     JacobiPreconditionerType, LeftILUT, PCGSolver, RightILUT, mvmult)

__all__ = ["Nonlinear", "AMG", "DefaultDirect", "RightIC", "GaussSeidelSmoother", "JacobiSmoother", "Linear", "CommonSolverArgs", "IterativeSolver", "NamedObject", "SolveStatus", "GMRES", "PCG",
           "GMRESSolver", "PCGSolver", "DeviceCSR", "DeviceVector", "IdentityPreconditioner",
           "IdentityPreconditionerType", "IterativeLinearSolver", "Jacobi", "JacobiPreconditioner",
           "JacobiPreconditionerType", "LeftILUT", "RightILUT", "mvmult"]
