"""slate_amd: MI355X-native distributed dense linear algebra.

A new implementation (not a port) of the capabilities of SLATE
(xiaohunqupo/slate): tiled distributed matrices over a 2D block-cyclic grid
of MI355X GPUs (one process per GPU, RCCL over xGMI), parallel BLAS-3,
Cholesky / LU / QR / LQ factorizations and solvers, least squares,
eigenvalue and singular value problems, norms and condition estimates,
with every hot kernel hand-written in HIP for CDNA4 (gfx950).

Public API mirrors `include/slate/slate.hh` and the simplified names of
`include/slate/simplified_api.hh`.
"""
__version__ = "2026.10.0"

from . import _native  # noqa: F401  (loads _host, tries _hip)
from .core.enums import (  # noqa: F401
    AllDevices, AnyDevice, Diag, Direction, Equed, GridOrder, HostNum, Job, Layout, LayoutConvert,
    MethodCholQR, MethodEig, MethodGels, MethodGemm, MethodHemm, MethodLU, MethodSVD, MethodTrsm,
    MOSI, Norm, NormScope, Op, Option, Side, Target, TileKind, Uplo)
from .core.exceptions import (  # noqa: F401
    CommError, HipError, NotImplementedYet, NumericalError, SlateError, slate_assert, slate_error,
    slate_error_if)
from .core.options import Options, get_option  # noqa: F401
from .core.tile import Tile  # noqa: F401
from .core.matrix import (  # noqa: F401
    BandMatrix, BaseBandMatrix, BaseMatrix, BaseTrapezoidMatrix, BaseTriangularBandMatrix,
    HermitianBandMatrix, HermitianMatrix, Matrix, Pivot, Pivots, SymmetricMatrix, TrapezoidMatrix,
    TriangularBandMatrix, TriangularFactors, TriangularMatrix)
from .core import func  # noqa: F401
from .parallel.comm import Comm, ProcessGrid, finalize, init, world  # noqa: F401
from .utils.matgen import MatgenParams, generate_matrix  # noqa: F401
from .utils.trace import Trace, trace_block  # noqa: F401
from .utils.timers import timers, timer  # noqa: F401
from .utils.watchdog import Watchdog  # noqa: F401

from .models.blas3 import (  # noqa: F401
    gemm, hemm, her2k, herk, multiply, rank_2k_update, rank_k_update, symm, syr2k, syrk,
    triangular_multiply, triangular_solve, trmm, trsm)
from .models.chol import posv, potrf, potri, potrs  # noqa: F401
from .models.aux import (  # noqa: F401
    add, allgather_dense, colNorms, copy, copy_conj_transpose, from_dense, gather, norm, redistribute, scale,
    scale_row_col, set)


def version():
    """SLATE `version()`: yyyymmdd-style integer."""
    return 20261015


def id():  # noqa: A001 - SLATE API name
    return "slate_amd-" + __version__


def chol_factor(A, opts=None):
    return potrf(A, opts)


def chol_solve(A, B, opts=None):
    return posv(A, B, opts)


def chol_solve_using_factor(A, B, opts=None):
    return potrs(A, B, opts)


def chol_inverse_using_factor(A, opts=None):
    return potri(A, opts)

from .models.lu import (  # noqa: F401,E402
    gesv, gesv_nopiv, getrf, getrf_nopiv, getrf_tntpiv, getri, getriOOP, getrs, getrs_nopiv, permute_rows)


def lu_factor(A, pivots, opts=None):
    return getrf(A, pivots, opts)


def lu_factor_nopiv(A, opts=None):
    return getrf_nopiv(A, opts)


def lu_solve(A, B, opts=None):
    return gesv(A, Pivots(), B, opts)


def lu_solve_nopiv(A, B, opts=None):
    return gesv_nopiv(A, B, opts)


def getrs_tntpiv(A, pivots, B, opts=None):
    """Solve with CALU factors (the pivots are an ordinary row permutation)."""
    return getrs(A, pivots, B, opts)


def lu_solve_using_factor(A, pivots, B, opts=None):
    return getrs(A, pivots, B, opts)


def lu_solve_using_factor_nopiv(A, B, opts=None):
    return getrs_nopiv(A, B, opts)


def lu_inverse_using_factor(A, pivots, opts=None):
    return getri(A, pivots, opts)


def lu_inverse_using_factor_out_of_place(A, pivots, B, opts=None):
    return getriOOP(A, pivots, B, opts)


from .models.qr import (  # noqa: F401,E402
    cholqr, gelqf, gels, gels_cholqr, gels_qr, geqrf, unmlq, unmqr)


def qr_factor(A, T, opts=None):
    return geqrf(A, T, opts)


def qr_multiply_by_q(side, op, A, T, C, opts=None):
    return unmqr(side, op, A, T, C, opts)


def lq_factor(A, T, opts=None):
    return gelqf(A, T, opts)


def lq_multiply_by_q(side, op, A, T, C, opts=None):
    return unmlq(side, op, A, T, C, opts)


def least_squares_solve(A, BX, opts=None):
    return gels(A, TriangularFactors(), BX, opts)


from .models.eig import (  # noqa: F401,E402
    eig, eig_vals, hb2st, he2hb, heev, hegst, hegv, stedc, stedc_deflate, stedc_secular, stedc_sort,
    stedc_z_vector, steqr, sterf, unmtr_hb2st, unmtr_he2hb)
from .models.svd import bdsqr, ge2tb, svd, svd_vals, tb2bd, unmbr_ge2tb, unmbr_tb2bd  # noqa: F401,E402


from .models.inverse import trtri, trtrm  # noqa: F401,E402
from .models.condest import gecondest, norm1est, pocondest, trcondest  # noqa: F401,E402
from .models.mixed import (  # noqa: F401,E402
    gerbt, gesv_mixed, gesv_mixed_gmres, gesv_rbt, posv_mixed, posv_mixed_gmres)


def lu_rcondest_using_factor(norm_type, A, pivots, anorm, opts=None):
    return gecondest(norm_type, A, pivots, anorm, opts)


def chol_rcondest_using_factor(norm_type, A, anorm, opts=None):
    return pocondest(norm_type, A, anorm, opts)


def triangular_rcondest(norm_type, A, anorm=None, opts=None):
    return trcondest(norm_type, A, anorm, opts)


from .models.band import (  # noqa: F401,E402
    band_mask, gbmm, gbsv, gbtrf, gbtrs, hbmm, pbsv, pbtrf, pbtrs, tbsm)
from .models.hetrf import hesv, hetrf, hetrs, sysv, sytrf, sytrs  # noqa: F401,E402


def indefinite_factor(A, pivots, T, pivots2, H, opts=None):
    return hetrf(A, pivots, T, pivots2, H, opts)


def indefinite_solve_using_factor(A, pivots, T, pivots2, B, opts=None):
    return hetrs(A, pivots, T, pivots2, B, opts)


def indefinite_solve(A, B, opts=None):
    return hesv(A, Pivots(), None, None, None, B, opts)


from .models.aux import set_lambda  # noqa: F401,E402


def gbnorm(norm_type, A, opts=None):
    """Norm of a general band matrix (computed from the in-band tiles)."""
    return norm(norm_type, A, opts)


def hbnorm(norm_type, A, opts=None):
    """Norm of a Hermitian band matrix (stored triangle + its reflection)."""
    return norm(norm_type, A, opts)
from .utils.printing import print_matrix, print_vector, format_matrix  # noqa: F401,E402
from .utils.debug import Debug  # noqa: F401,E402
from .models.svd import ge2tb as ge2tb_, svd_vals  # noqa: F401,E402
from . import compat  # noqa: F401,E402
print = print_matrix  # SLATE slate::print(label, A, opts)  # noqa: A001
