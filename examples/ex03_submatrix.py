"""ex03: sub-matrices and slices, transposes (reference ex03_submatrix.cc)."""
import slate_amd as sl

sl.init()
A = sl.Matrix(1000, 800, nb=100)
A.insertLocalTiles()
sl.generate_matrix(A, "ij", 0)
B = A.sub(2, 4, 1, 3)            # tiles (2..4) x (1..3)
C = A.slice(150, 449, 20, 219)   # elements
AT = A.transpose()
AH = A.conj_transpose()
if sl.world().rank == 0:
    print("ex03:", B.m(), B.n(), C.m(), C.n(), AT.m(), AT.n(), AH.op())
sl.finalize()
