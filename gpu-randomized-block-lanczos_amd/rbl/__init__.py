"""rbl — MI355X-native Randomized Block Lanczos inner loop (host side).

``RBL_gpu(A, k, b)`` mirrors Julia/RBL_gpu.jl:205; ``Context`` wraps the C-ABI of
librbl_hip.so (include/rbl_hip.h).  Importing this package loads the HIP library and fails
loudly if it has not been built: there is no CPU fallback.
"""
from ._lib import RBLError, lib, stage_names  # noqa: F401  (raises ImportError if unbuilt)
from .host import TBand, check_convergence, dsbev, sort_eig_abs  # noqa: F401
from . import io  # noqa: F401
from .restarted import RBL_gpu_restarted, RBL_restarted  # noqa: F401
from .rbl_gpu import (KRYL_SZ_GPU, RESIDUAL_TOL, Context, RBL_gpu, RBLInfo, LocalGroup,  # noqa: F401
                      lanczos, rccl_version)
