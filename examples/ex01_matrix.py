"""ex01: creating distributed matrices (reference examples/ex01_matrix.cc)."""
import torch
import slate_amd as sl

sl.init()
comm = sl.world()
p, q = (2, comm.size // 2) if comm.size % 2 == 0 and comm.size > 1 else (1, comm.size)
dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
# empty matrix with 2D block-cyclic tiles, then allocate local tiles on the GPU (or host)
A = sl.Matrix(2000, 1000, nb=256, p=p, q=q, device=dev)
A.insertLocalTiles(device=0 if dev is not None else -1)
sl.generate_matrix(A, "rands", seed=42)
# wrap an existing column-major (LAPACK) array, replicated on every rank
X = torch.randn(300, 200, dtype=torch.float64).t().contiguous().t()
B = sl.Matrix.fromLAPACK(300, 200, X, X.stride(1), nb=64)
# typed views
H = sl.HermitianMatrix(sl.Uplo.Lower, 500, nb=128, p=p, q=q, device=dev)
T = sl.TriangularMatrix(sl.Uplo.Upper, sl.Diag.Unit, A.sub(0, 1, 0, 1)) if False else None
if comm.rank == 0:
    print("ex01:", A, B, H, sep="\n  ")
sl.finalize()
