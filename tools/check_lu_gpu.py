import sys, torch, time
sys.path.insert(0, '.')
import slate_amd as sl
from slate_amd.models.aux import allgather_dense as D
dev = torch.device('cuda')
for n, nb in [(1000, 128), (4096, 512)]:
    A = sl.Matrix(n, n, nb=nb, device=dev); A.insertLocalTiles(device=dev); sl.generate_matrix(A, 'rands', 5)
    A0 = D(A).double()
    piv = sl.Pivots()
    t0 = time.perf_counter(); info = sl.getrf(A, piv); torch.cuda.synchronize(); t = time.perf_counter() - t0
    B = sl.Matrix(n, 3, nb=nb, device=dev); B.insertLocalTiles(device=dev); sl.generate_matrix(B, 'rands', 6)
    B0 = D(B)
    sl.getrs(A, piv, B)
    X = D(B)
    res = ((A0 @ X - B0).abs().max() / (A0.abs().max() * X.abs().max() * n)).item()
    print(f"getrf n={n} nb={nb} info={info} t={t*1e3:.1f} ms backward_err={res:.2e}", flush=True)
