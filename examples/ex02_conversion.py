"""ex02: conversions between matrix types (reference ex02_conversion.cc)."""
import slate_amd as sl

sl.init()
A = sl.Matrix(400, 400, nb=100)
A.insertLocalTiles()
sl.generate_matrix(A, "rands", 1)
L = sl.TriangularMatrix(sl.Uplo.Lower, sl.Diag.NonUnit, A)      # shallow view of the lower triangle
H = sl.HermitianMatrix(sl.Uplo.Lower, A)                         # Hermitian view
S = sl.SymmetricMatrix(sl.Uplo.Upper, A)
Z = A.emptyLike()                                                  # same distribution, no data
if sl.world().rank == 0:
    print("ex02:", L, H, S, Z, sep="\n  ")
sl.finalize()
