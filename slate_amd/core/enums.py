"""Enumerations of the public API.

Names and character codes mirror SLATE's `include/slate/enums.hh:38-543`
(Target, Method*, Option, LayoutConvert, NormScope, GridOrder, MOSI) and the
BLAS++/LAPACK++ enums SLATE re-exports (Op, Uplo, Diag, Side, Layout, Norm,
Job, ...), so code written against the reference maps 1:1.

MI355X note: ``Target.Devices`` means "this rank's MI355X" -- one process
drives one GPU (rank == GPU); there is no per-rank device list.
"""
from __future__ import annotations

import enum


class _CharEnum(str, enum.Enum):
    def __str__(self):
        return self.value

    @classmethod
    def from_string(cls, s):
        """Case-insensitive lookup by name or character code."""
        if isinstance(s, cls):
            return s
        key = str(s).strip()
        for m in cls:
            if m.value == key or m.name.lower() == key.lower():
                return m
        for m in cls:
            if m.value.lower() == key.lower():
                return m
        raise ValueError(f"invalid {cls.__name__}: {s!r}")

    def to_string(self):
        return self.name


class Target(_CharEnum):
    """Where/how computation runs (`enums.hh:38-44`)."""
    Host = 'H'
    HostTask = 'T'
    HostNest = 'N'
    HostBatch = 'B'
    Devices = 'D'


class MethodTrsm(_CharEnum):
    Auto = '*'
    A = 'A'     # stationary A (reduce-based)
    B = 'B'     # stationary B


class MethodGemm(_CharEnum):
    Auto = '*'
    A = 'A'     # stationary A, reduce partial C
    C = 'C'     # stationary C (SUMMA)


class MethodHemm(_CharEnum):
    Auto = '*'
    A = 'A'
    C = 'C'


class MethodCholQR(_CharEnum):
    Auto = '*'
    GemmA = 'A'
    GemmC = 'C'
    HerkA = 'R'
    HerkC = 'K'


class MethodGels(_CharEnum):
    Auto = '*'
    QR = 'Q'
    CholQR = 'C'


class MethodLU(_CharEnum):
    Auto = '*'
    PartialPiv = 'P'
    CALU = 'C'
    NoPiv = 'N'
    RBT = 'R'
    BEAM = 'B'


class MethodEig(_CharEnum):
    Auto = '*'
    QR = 'Q'
    DC = 'D'
    Bisection = 'B'
    MRRR = 'M'


class MethodSVD(_CharEnum):
    Auto = '*'
    QR = 'Q'
    DC = 'D'
    Bisection = 'B'


class Option(enum.IntEnum):
    """Keys of the per-call options map (`enums.hh:461-498`)."""
    ChunkSize = 0
    Lookahead = 1
    BlockSize = 2
    InnerBlocking = 3
    MaxPanelThreads = 4
    Tolerance = 5
    Target = 6
    HoldLocalWorkspace = 7
    Depth = 8
    MaxIterations = 9
    UseFallbackSolver = 10
    PivotThreshold = 11
    PrintVerbose = 50
    PrintEdgeItems = 51
    PrintWidth = 52
    PrintPrecision = 53
    MethodCholQR = 60
    MethodEig = 61
    MethodGels = 62
    MethodGemm = 63
    MethodHemm = 64
    MethodLU = 65
    MethodTrsm = 66
    MethodSVD = 67
    # MI355X extensions
    UseGraph = 100        # capture the factorization DAG into a hipGraph
    PanelStreamPriority = 101


class LayoutConvert(_CharEnum):
    ColMajor = 'C'
    RowMajor = 'R'
    None_ = 'N'


class NormScope(_CharEnum):
    Columns = 'C'
    Rows = 'R'
    Matrix = 'M'


class GridOrder(_CharEnum):
    Col = 'C'
    Row = 'R'
    Unknown = 'U'


HostNum = -1
AllDevices = -2
AnyDevice = -3


class MOSI(enum.IntFlag):
    """Tile-instance coherency states (`enums.hh:537-543`)."""
    Invalid = 0x001
    Shared = 0x010
    Modified = 0x100
    OnHold = 0x1000


class TileKind(enum.IntEnum):
    """`include/slate/Tile.hh:97-101`."""
    Workspace = 0
    SlateOwned = 1
    UserOwned = 2


# ---- BLAS/LAPACK enums (re-exported by SLATE from BLAS++/LAPACK++) -------
class Op(_CharEnum):
    NoTrans = 'N'
    Trans = 'T'
    ConjTrans = 'C'


class Uplo(_CharEnum):
    Upper = 'U'
    Lower = 'L'
    General = 'G'


class Diag(_CharEnum):
    NonUnit = 'N'
    Unit = 'U'


class Side(_CharEnum):
    Left = 'L'
    Right = 'R'


class Layout(_CharEnum):
    ColMajor = 'C'
    RowMajor = 'R'


class Norm(_CharEnum):
    One = '1'
    Two = '2'
    Inf = 'I'
    Fro = 'F'
    Max = 'M'


class Job(_CharEnum):
    NoVec = 'N'
    Vec = 'V'
    Update = 'U'
    AllVec = 'A'
    SomeVec = 'S'
    OverwriteVec = 'O'
    CompactVec = 'P'
    SomeVecTol = 'C'
    VecJacobi = 'J'
    Workspace = 'W'


class Direction(_CharEnum):
    Forward = 'F'
    Backward = 'B'


class Equed(_CharEnum):
    None_ = 'N'
    Row = 'R'
    Col = 'C'
    Both = 'B'


def transpose_op(op: Op) -> Op:
    return Op.NoTrans if op != Op.NoTrans else Op.Trans


def conj_transpose_op(op: Op) -> Op:
    return Op.NoTrans if op != Op.NoTrans else Op.ConjTrans
