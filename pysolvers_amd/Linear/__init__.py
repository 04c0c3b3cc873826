"""Drop-in for PySolvers.Linear's PCG/GMRES path (Linear/__init__.py:1-12 names)."""
from .DeviceMatrix import DeviceCSR, DeviceVector, spmv
from .GMRESSolver import GMRES, GMRESSolver
from .ILUTPreconditioner import (ILUTPreconditioner, LeftILUT, LeftILUTPreconditioner, RightILUT,
                                 RightILUTPreconditioner)
from .IterativeLinearSolver import IterativeLinearSolver, IterativeLinearSolverType, mvmult
from .LinearSolver import LinearSolver, LinearSolverType
from .PCGSolver import PCG, PCGSolver
from .Preconditioner import (GenericPreconditioner, IdentityPreconditioner, JacobiPreconditioner,
                             LeftPreconditioner, Preconditioner, RightPreconditioner)
from .PreconditionerType import (IdentityPreconditionerType, Jacobi, JacobiPreconditionerType,
                                 PreconditionerType)
