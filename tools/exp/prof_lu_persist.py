"""Per-phase clocks of the persistent LU base case (workgroup 0), standalone
panel and inside the dgetrf bench factorization."""
import time, torch
from slate_amd import ops, _native
H = _native.hip()
PH = ["local arg-max", "publish+drain", "arrive+poll", "gather+argmax", "swap+elim"]
def report(tag, cols):
    v = H.lu_persist_profile(0)
    tot = sum(v[:5])
    print(f"{tag}: {cols} columns, {tot / cols / 2.4e3:.2f} us/column at 2.4 GHz: " +
          ", ".join(f"{PH[k]} {v[k] / cols / 2.4e3:.2f}" for k in range(5)), flush=True)
m, n = 32768, 512
g = torch.Generator().manual_seed(1)
A0 = torch.randn(m, n, dtype=torch.float64, generator=g).t().contiguous().t().cuda()
ipiv = torch.zeros(n, dtype=torch.int64, device="cuda")
A = A0.clone(); ops.getrf(A, ipiv); torch.cuda.synchronize()
H.lu_persist_profile(1)
A = A0.clone(); ops.getrf(A, ipiv); torch.cuda.synchronize()
report("standalone panel 32768x512", n)
import subprocess, sys
import slate_amd as sl
dev = torch.device("cuda", 0)
N = 32768
M = sl.Matrix(N, N, nb=512, p=1, q=1, device=dev)
M.insertLocalTiles(device=dev)
sl.generate_matrix(M, "rands", seed=7)
piv = sl.Pivots()
opts = {sl.Option.Lookahead: 2, sl.Option.Target: sl.Target.Devices}
H.lu_persist_profile(1)
t0 = time.perf_counter(); sl.getrf(M, piv, opts); torch.cuda.synchronize(); dt = time.perf_counter() - t0
report(f"inside dgetrf n={N} ({dt * 1e3:.0f} ms)", N)
