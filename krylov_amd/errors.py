class ArgumentError(Exception):
    """Raised when an argument is invalid, e.g. iterating on an invariant
    Krylov space (mirrors ``krylov.errors.ArgumentError``, errors.py:1-9)."""

    def __init__(self, message):
        super().__init__(message)
