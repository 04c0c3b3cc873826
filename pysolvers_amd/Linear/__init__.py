"""Drop-in for PySolvers.Linear's PCG/GMRES path (Linear/__init__.py:1-12 names)."""
from .AMGPreconditioner import AMG, AMGPreconditioner
from .ClassicSmoothers import GaussSeidelSmoother, JacobiSmoother
from .DeviceMatrix import DeviceCSR, DeviceVector, spmv
from .DirectSolver import DefaultDirect, DefaultDirectSolver
from .Distributed import Communicator, fd_laplacian_2d_sharded, halo_cols, shard_csr
from .GMRESSolver import GMRES, GMRESSolver
from .ILUTPreconditioner import (ILUTPreconditioner, LeftILUT, LeftILUTPreconditioner, RightILUT,
                                 RightILUTPreconditioner)
from .ICPreconditioner import ICRightPreconditioner, RightIC
from .IterativeLinearSolver import IterativeLinearSolver, IterativeLinearSolverType, mvmult
from .LinearSolver import LinearSolver, LinearSolverType
from .PCGSolver import PCG, PCGSolver
from .MLHierarchy import MLHierarchy, makeRestrictionOp
from .Preconditioner import (DeviceOperator, GenericPreconditioner, IdentityPreconditioner, JacobiPreconditioner,
                             LeftPreconditioner, Preconditioner, RightPreconditioner)
from .PreconditionerType import (IdentityPreconditionerType, Jacobi, JacobiPreconditionerType,
                                 PreconditionerType)
from .SmoothedAggregation import SA_coarsen, SmoothedAggregationMLHierarchy
from .TriangularSolve import TriangularSolveChain
