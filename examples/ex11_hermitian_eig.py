"""ex11: Hermitian eigenvalues/vectors (reference ex11_hermitian_eig.cc)."""
import slate_amd as sl

sl.init()
n, nb = 500, 64
A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb)
Z = sl.Matrix(n, n, nb=nb)
for M in (A, Z):
    M.insertLocalTiles()
sl.generate_matrix(A, "rands", 1)
w = sl.eig(A, None, Z)                        # heev (2-stage) with eigenvectors
if sl.world().rank == 0:
    print("ex11: lambda range", float(w[0]), float(w[-1]))
sl.finalize()
