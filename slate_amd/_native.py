"""Loader for the native extensions and the tensor -> kernel-module dispatch.

``_hip`` (gfx950 kernels) is REQUIRED whenever a tensor lives on a GPU: if
it is missing or fails to load, GPU calls raise instead of silently falling
back to PyTorch/vendor code.  ``_host`` (native host runtime + CPU tile
kernels) is required always.
"""
from __future__ import annotations

import os

import torch

from .core.exceptions import HipError

_host_override = os.environ.get("SLATE_AMD_HOST_LIB")    # e.g. the sanitizer build (tools/asan)
try:
    if _host_override:
        import importlib.util as _ilu
        _spec = _ilu.spec_from_file_location("slate_amd._host", _host_override)
        _host = _ilu.module_from_spec(_spec)
        _spec.loader.exec_module(_host)
    else:
        from . import _host  # noqa: F401
except ImportError as e:  # pragma: no cover - build problem
    raise ImportError(
        "slate_amd._host is not built; run `python slate_amd/_build.py` "
        f"(or __graft_entry__.build()): {e}") from e

_hip = None
_hip_error = None
try:
    from . import _hip  # noqa: F811
except Exception as e:  # noqa: BLE001
    _hip_error = e

DTYPE_CODE = {
    torch.float32: 's',
    torch.float64: 'd',
    torch.complex64: 'c',
    torch.complex128: 'z',
}
CODE_DTYPE = {v: k for k, v in DTYPE_CODE.items()}
REAL_OF = {torch.float32: torch.float32, torch.float64: torch.float64,
           torch.complex64: torch.float32, torch.complex128: torch.float64}


def hip():
    if _hip is None:
        raise HipError(f"slate_amd._hip (gfx950 kernels) failed to load: {_hip_error!r}; "
                       "build it with `python slate_amd/_build.py`")
    return _hip


def kmod(t: torch.Tensor):
    """Kernel module for the memory space of tensor t."""
    return hip() if t.is_cuda else _host


def stream(t: torch.Tensor | None = None) -> int:
    if t is not None and not t.is_cuda:
        return 0
    if not torch.cuda.is_available():
        return 0
    return torch.cuda.current_stream().cuda_stream


def code(dtype) -> str:
    try:
        return DTYPE_CODE[dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {dtype}") from None


def hip_available() -> bool:
    return _hip is not None and torch.cuda.is_available()


def loaded_native_modules():
    mods = [_host.__file__]
    if _hip is not None:
        mods.append(_hip.__file__)
    return [os.path.abspath(m) for m in mods]
