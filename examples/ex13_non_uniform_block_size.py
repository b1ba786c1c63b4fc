"""ex13: non-uniform tile sizes via the lambda constructor (reference ex13_non_uniform_block_size.cc)."""
import slate_amd as sl

sl.init()
comm = sl.world()
sizes = [100, 200, 50, 150]                   # tile rows/cols
m = n = sum(sizes)
def tile_mb(i): return sizes[i % len(sizes)]
def tile_rank(ij): return (ij[0] + ij[1]) % comm.size
A = sl.Matrix.from_functions(m, n, tile_mb, tile_mb, tile_rank)
A.insertLocalTiles()
sl.generate_matrix(A, "rands", 1)
nrm = float(sl.norm(sl.Norm.Fro, A))
if comm.rank == 0:
    print("ex13:", A, nrm)
sl.finalize()
