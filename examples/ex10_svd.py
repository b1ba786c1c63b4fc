"""ex10: singular value decomposition (reference ex10_svd.cc)."""
import slate_amd as sl

sl.init()
m, n, nb = 500, 300, 64
A = sl.Matrix(m, n, nb=nb)
U, VH = sl.Matrix(m, n, nb=nb), sl.Matrix(n, n, nb=nb)
for M in (A, U, VH):
    M.insertLocalTiles()
sl.generate_matrix(A, "rands", 1)
s = sl.svd(A, None, U, VH)
if sl.world().rank == 0:
    print("ex10: sigma_max", float(s[0]), "sigma_min", float(s[-1]))
sl.finalize()
