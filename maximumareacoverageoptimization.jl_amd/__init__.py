"""MI355X-native MADS area-coverage objective (Gabisanth/MaximumAreaCoverageOptimization.jl).

The product is libmaxcover.so (HIP kernels for gfx950 + the C-ABI in include/maxcover.h); this
package is the host-side mirror of the reference's Julia modules on the hot path, binding the
library through ctypes. Loading the package does not touch the GPU; the first evaluation
creates a context (and fails loudly if the library or a GPU is missing).
"""
from ._lib import (ALGOS, Context, Fire, InexactError, MaxCoverError, cover_threshold,
                   default_context, device_count, load_library, version)
from . import Base_Functions, firepoints, workloads  # noqa: F401  (pure host modules)
from . import AreaCoverageCalculation, CellFunctions, DynamicArea, TDM_Constraints  # noqa: F401
from . import FullSimulation, TDM_STATIC_opt  # noqa: F401

__all__ = ["ALGOS", "Context", "Fire", "InexactError", "MaxCoverError", "cover_threshold",
           "default_context", "device_count", "load_library", "version",
           "AreaCoverageCalculation", "CellFunctions", "DynamicArea", "FullSimulation",
           "TDM_Constraints",
           "TDM_STATIC_opt", "Base_Functions", "firepoints", "workloads"]
