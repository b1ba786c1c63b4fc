"""ex07: Cholesky solve, mixed precision (reference ex07_linear_system_cholesky.cc)."""
import slate_amd as sl

sl.init()
n, nrhs, nb = 600, 3, 128
A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb)
B, X = sl.Matrix(n, nrhs, nb=nb), sl.Matrix(n, nrhs, nb=nb)
for M in (A, B, X):
    M.insertLocalTiles()
sl.generate_matrix(A, "poev", 1)
sl.generate_matrix(B, "rands", 2)
info, iters = sl.posv_mixed(A, B, X)          # fp32 Cholesky + fp64 refinement
info2 = sl.chol_solve(A, B)                   # potrf + potrs
if sl.world().rank == 0:
    print("ex07: info", info, "IR iterations", iters, info2)
sl.finalize()
