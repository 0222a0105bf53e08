"""Exceptions of the device path and the mapping from C-ABI status codes.

``ArgumentError`` keeps the reference's name and role (``krylov.errors``,
errors.py:1-9): iterating an invariant Krylov space raises it
(arnoldi.py:67-70, 168-171, 239-242). The other statuses that
``libkrylov_hip.so`` returns (include/krylov_hip.h, ``KRY_E*``) map to the
built-in exceptions the reference's NumPy/SciPy calls would raise at the same
point.
"""
import numpy as np


class ArgumentError(Exception):
    """Invalid argument in the Krylov sense: the space became invariant."""


# KRY_E* status -> exception type (include/krylov_hip.h "status codes")
STATUS_EXCEPTIONS = {
    -1: ValueError,                 # KRY_EINVAL: shape / dtype / handle
    -2: MemoryError,                # KRY_ENOMEM: device allocation
    -3: RuntimeError,               # KRY_EDEVICE: HIP runtime, no device
    -4: ArgumentError,              # KRY_EINVARIANT: arnoldi.py:168-171
    -5: NotImplementedError,        # KRY_EUNSUPPORTED: outside the device path
    -6: np.linalg.LinAlgError,      # KRY_ESINGULAR: solve_triangular (gmres.py:36)
    -7: ValueError,                 # KRY_ENONFINITE: NaN/inf into solve_triangular
    -8: RuntimeError,               # KRY_ECOMM: RCCL
}


def exception_for(status, message):
    """The exception instance for a non-zero C-ABI status."""
    exc = STATUS_EXCEPTIONS.get(status)
    if exc is None:
        return RuntimeError(f"libkrylov_hip error {status}: {message}")
    if exc is RuntimeError:
        return RuntimeError(f"libkrylov_hip error {status}: {message}")
    return exc(message)
