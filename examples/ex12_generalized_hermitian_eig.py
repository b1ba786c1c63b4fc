"""ex12: generalized Hermitian-definite eigenproblem (reference ex12_generalized_hermitian_eig.cc)."""
import slate_amd as sl

sl.init()
n, nb = 300, 64
A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb)
B = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb)
Z = sl.Matrix(n, n, nb=nb)
for M in (A, B, Z):
    M.insertLocalTiles()
sl.generate_matrix(A, "rands", 1)
sl.generate_matrix(B, "poev", 2)
w = sl.hegv(1, A, B, None, Z)                 # A z = lambda B z
if sl.world().rank == 0:
    print("ex12: lambda range", float(w[0]), float(w[-1]))
sl.finalize()
