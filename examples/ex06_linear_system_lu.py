"""ex06: LU solve (reference ex06_linear_system_lu.cc)."""
import slate_amd as sl

sl.init()
n, nrhs, nb = 600, 5, 128
A, B = sl.Matrix(n, n, nb=nb), sl.Matrix(n, nrhs, nb=nb)
for i, M in enumerate((A, B)):
    M.insertLocalTiles()
    sl.generate_matrix(M, "rands", i)
piv = sl.Pivots()
info = sl.lu_solve(A, B)                      # getrf + getrs
A2 = sl.Matrix(n, n, nb=nb)
A2.insertLocalTiles()
sl.generate_matrix(A2, "rands", 0)
info2 = sl.lu_factor(A2, piv)
inv_info = sl.lu_inverse_using_factor(A2, piv)
if sl.world().rank == 0:
    print("ex06: info", info, info2, inv_info)
sl.finalize()
