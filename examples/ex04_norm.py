"""ex04: matrix norms (reference ex04_norm.cc)."""
import slate_amd as sl

sl.init()
A = sl.Matrix(500, 300, nb=64)
A.insertLocalTiles()
sl.generate_matrix(A, "rands", 3)
vals = {n: float(sl.norm(n, A)) for n in (sl.Norm.Max, sl.Norm.One, sl.Norm.Inf, sl.Norm.Fro)}
if sl.world().rank == 0:
    print("ex04:", {k.name: round(v, 4) for k, v in vals.items()})
sl.finalize()
