"""ex14: ScaLAPACK-style gemm on this rank's local arrays (reference ex14_scalapack_gemm.cc)."""
import numpy as np
import slate_amd as sl
from slate_amd.compat import scalapack as S

sl.init()
comm = sl.world()
p, q = 1, comm.size
ctxt = S.blacs_gridinit(p, q)
_, _, pr, pc = S.blacs_gridinfo(ctxt)
m = n = k = 256
nb = 64
mloc, nloc = S.numroc(m, nb, pr, 0, p), S.numroc(n, nb, pc, 0, q)
A = np.asfortranarray(np.random.default_rng(1).standard_normal((mloc, nloc)))
B = np.asfortranarray(np.random.default_rng(2).standard_normal((mloc, nloc)))
C = np.zeros((mloc, nloc), order="F")
desc = [1, ctxt, m, n, nb, nb, 0, 0, max(1, mloc)]
S.pdgemm('N', 'N', m, n, k, 1.0, A, 1, 1, desc, B, 1, 1, desc, 0.0, C, 1, 1, desc)
if comm.rank == 0:
    print("ex14: local C norm", float(np.linalg.norm(C)))
sl.finalize()
