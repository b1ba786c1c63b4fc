"""ex05: parallel BLAS-3 (reference ex05_blas.cc)."""
import slate_amd as sl

sl.init()
m, n, k, nb = 400, 300, 200, 64
A, B, C = (sl.Matrix(*d, nb=nb) for d in ((m, k), (k, n), (m, n)))
for i, M in enumerate((A, B, C)):
    M.insertLocalTiles()
    sl.generate_matrix(M, "rands", i)
sl.gemm(1.0, A, B, 0.5, C)                                        # C = A B + C/2
Hc = sl.HermitianMatrix(sl.Uplo.Lower, m, nb=nb)
Hc.insertLocalTiles()
sl.herk(1.0, A, 0.0, Hc)                                          # Hc = A A^H
T = sl.TriangularMatrix(sl.Uplo.Lower, sl.Diag.Unit, sl.Matrix(m, m, nb=nb))
T.insertLocalTiles()
sl.generate_matrix(T, "rands", 7)
sl.trsm(sl.Side.Left, 1.0, T, C)                                  # C = T^{-1} C
sl.trmm(sl.Side.Left, 1.0, T, C)                                  # C = T C
sl.multiply(1.0, A, B, 0.0, C)                                    # simplified API names
nrm = float(sl.norm(sl.Norm.Fro, C))             # collective: every rank calls it
if sl.world().rank == 0:
    print("ex05: ok", nrm)
sl.finalize()
