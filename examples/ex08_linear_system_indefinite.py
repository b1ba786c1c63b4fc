"""ex08: Hermitian indefinite solve (reference ex08_linear_system_indefinite.cc)."""
import slate_amd as sl

sl.init()
n, nb = 400, 64
A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb)
B = sl.Matrix(n, 2, nb=nb)
for M in (A, B):
    M.insertLocalTiles()
sl.generate_matrix(A, "rands", 1)
sl.generate_matrix(B, "rands", 2)
info = sl.indefinite_solve(A, B)              # hetrf + hetrs
if sl.world().rank == 0:
    print("ex08: info", info)
sl.finalize()
