"""krylov_amd — MI355X-native inner loop for the Krylov solvers of
``ju-liu/krylov`` (cg / gmres / minres with the reference call signatures;
bicgstab / cgs / cgr / gcr with their scalars chained on the device, over the
same kernels).

The per-iteration work (CSR SpMV, AXPY/scale updates, inner products and
norms, GMRES modified Gram-Schmidt + Givens, the MINRES Lanczos/QR
recurrences) runs as hand-written gfx950 HIP kernels in ``libkrylov_hip.so``
reached through a ctypes C-ABI (``include/krylov_hip.h``). There is no CPU
fallback: importing this package without the built library raises.
"""
from ._helpers import Identity, Info, WeightedInner, aslinearoperator, get_default_inner
from .cg import cg
from .errors import ArgumentError
from .extra import bicgstab, cgr, cgs, gcr
from .givens import givens, lartg
from .householder import Householder
from .gmres import arnoldi, gmres, gmres_restarted, multi_solve_triangular
from .minres import lanczos, minres
from ._lib import empty_cache, memory_stats
from .sparse import CsrOperator, as_device_operator, clear_operator_cache

__version__ = "0.1.0"

__all__ = [
    "cg",
    "gmres",
    "gmres_restarted",
    "multi_solve_triangular",
    "arnoldi",
    "lanczos",
    "minres",
    "bicgstab",
    "cgs",
    "cgr",
    "gcr",
    "givens",
    "Householder",
    "lartg",
    "CsrOperator",
    "as_device_operator",
    "clear_operator_cache",
    "memory_stats",
    "empty_cache",
    "WeightedInner",
    "Identity",
    "Info",
    "aslinearoperator",
    "get_default_inner",
    "ArgumentError",
    "__version__",
]
