"""ex15: setting matrix entries with a function of (i, j) (reference ex15_set_matrix.cc)."""
import slate_amd as sl

sl.init()
A = sl.Matrix(300, 200, nb=64)
A.insertLocalTiles()
sl.set_lambda(lambda i, j: 1.0 / (i + j + 1.0), A)    # Hilbert matrix
sl.set(0.0, 1.0, A.slice(0, 9, 0, 9))                  # identity block
# print is collective (gathers to rank 0, which prints)
sl.print("A", A.slice(0, 11, 0, 5), {sl.Option.PrintVerbose: 4, sl.Option.PrintPrecision: 3})
sl.finalize()
