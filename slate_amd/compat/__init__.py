"""Compatibility front-ends: LAPACK-style (`lapack`),
ScaLAPACK-style (`scalapack`) routines, and the C ABI (csrc/capi ->
libslate_amd_c.so, header include/slate_amd/c_api.h)."""
from . import lapack, scalapack  # noqa: F401
