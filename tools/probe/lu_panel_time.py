"""Latency of the fp64 LU panel (ops.getrf on an m x 512 block) for the
heights the dgetrf n = 32768 factorization walks through, standalone on an
idle GPU; plus the per-phase clocks of the persistent base case."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from slate_amd import ops, _native

H = _native.hip()
PH = ["local arg-max", "publish+drain", "arrive+poll", "gather+argmax", "swap+elim"]
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 512
g = torch.Generator().manual_seed(1)
for m in (32768, 24576, 16384, 8192, 4096, 2048, 1024):
    A0 = torch.randn(m, nb, dtype=torch.float64, generator=g).t().contiguous().t().cuda()
    ipiv = torch.zeros(nb, dtype=torch.int64, device="cuda")
    ts = []
    for it in range(6):
        A = A0.clone()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.getrf(A, ipiv)
        e1.record()
        torch.cuda.synchronize()
        if it:
            ts.append(e0.elapsed_time(e1))
    ts.sort()
    H.lu_persist_profile(1)
    A = A0.clone(); ops.getrf(A, ipiv); torch.cuda.synchronize()
    v = H.lu_persist_profile(0)
    ph = ", ".join(f"{PH[k]} {v[k] / nb / 2.4e3:.2f}" for k in range(5))
    # check: P A = L U
    L = torch.tril(A, -1)[:, :nb] + torch.eye(m, nb, dtype=A.dtype, device=A.device)
    U = torch.triu(A[:nb])
    PA = A0.clone()
    for j in range(nb):
        p = int(ipiv[j])
        if p != j:
            PA[[j, p]] = PA[[p, j]]
    err = ((PA - L @ U).norm() / A0.norm()).item()
    print(f"m={m:6d} n={nb}: {ts[len(ts) // 2]:.3f} ms median ({ts[len(ts) // 2] / nb * 1e3:.2f} us/col) "
          f"err {err:.1e} | phases us/col: {ph}", flush=True)
