"""Error types and checking helpers (`include/slate/Exception.hh:10-101`,
`include/slate/internal/mpi.hh:17-53`).

`hip_call` / `comm_call` replace SLATE's `slate_mpi_call`: they wrap a native
or collective call and re-raise failures with the call site attached.
"""
from __future__ import annotations

import functools
import inspect


class SlateError(RuntimeError):
    """Base class of all errors raised by slate_amd (SLATE `Exception`)."""

    def __init__(self, msg="", func=None, file=None, line=None):
        if func is None:
            fr = inspect.stack()[1]
            func, file, line = fr.function, fr.filename, fr.lineno
        self.func, self.file, self.line = func, file, line
        super().__init__(f"{msg}, in function {func} at {file}:{line}" if msg else
                         f"error in function {func} at {file}:{line}")


class NotImplementedYet(SlateError, NotImplementedError):
    """SLATE `NotImplemented`."""


class CommError(SlateError):
    """Failure of a collective / point-to-point transfer (SLATE `MpiException`)."""


class HipError(SlateError):
    """Failure reported by the HIP runtime or a kernel launch."""


class NumericalError(SlateError):
    """A factorization reported info > 0 and the caller asked for an exception."""

    def __init__(self, msg, info):
        self.info = info
        super().__init__(msg)


def slate_error(msg):
    raise SlateError(msg)


def slate_error_if(cond, msg="condition failed"):
    if cond:
        fr = inspect.stack()[1]
        raise SlateError(f"{msg}", fr.function, fr.filename, fr.lineno)


def slate_assert(cond, msg="assertion failed"):
    if not cond:
        fr = inspect.stack()[1]
        raise SlateError(f"{msg}", fr.function, fr.filename, fr.lineno)


def comm_call(fn):
    """Decorator: wrap collective failures into CommError."""
    @functools.wraps(fn)
    def wrapper(*a, **k):
        try:
            return fn(*a, **k)
        except SlateError:
            raise
        except Exception as e:  # noqa: BLE001
            raise CommError(f"{fn.__name__}: {e}") from e
    return wrapper
