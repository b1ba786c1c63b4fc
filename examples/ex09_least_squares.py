"""ex09: least squares, QR / CholeskyQR (reference ex09_least_squares.cc)."""
import slate_amd as sl

sl.init()
m, n, nb = 900, 300, 128
A, BX = sl.Matrix(m, n, nb=nb), sl.Matrix(m, 2, nb=nb)
for i, M in enumerate((A, BX)):
    M.insertLocalTiles()
    sl.generate_matrix(M, "rands", i)
sl.least_squares_solve(A, BX)                # geqrf + unmqr + trsm; X = BX[0:n, :]
A2, B2 = sl.Matrix(m, n, nb=nb), sl.Matrix(m, 2, nb=nb)
for i, M in enumerate((A2, B2)):
    M.insertLocalTiles()
    sl.generate_matrix(M, "rands", i)
sl.gels_cholqr(A2, B2)
if sl.world().rank == 0:
    print("ex09: ok")
sl.finalize()
