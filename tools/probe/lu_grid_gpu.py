"""Probe: distributed getrf on one GPU with 4 gloo ranks, pipelined vs serial streams."""
import os, sys, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import slate_amd as sl
from slate_amd.core.enums import Option
from dist_util import run_dist


def f(rank, size, p, q, la, n, nb, serial):
    os.environ["SLATE_AMD_SERIAL"] = serial
    torch.cuda.set_device(0)
    from slate_amd.models.aux import allgather_dense as D
    A = sl.Matrix(n, n, nb=nb, p=p, q=q, device="cuda"); A.insertLocalTiles(device=0); sl.generate_matrix(A, "rands", 4)
    A0 = D(A); piv = sl.Pivots()
    info = sl.getrf(A, piv, {Option.Lookahead: la})
    F = D(A); L = torch.tril(F, -1) + torch.eye(n, dtype=F.dtype, device=F.device); perm = list(range(n))
    for i, pv in enumerate(piv.ipiv.tolist()): perm[i], perm[pv] = perm[pv], perm[i]
    r = ((L @ torch.triu(F) - A0[torch.as_tensor(perm, device=F.device)]).norm() / A0.norm()).item()
    from slate_amd import _native
    fb = _native.hip().lu_persist_fallbacks()
    print(f"grid {p}x{q} la={la} serial={serial} persist={os.environ.get('SLATE_AMD_LU_PERSIST','1')} "
          f"rank={rank} info={info} resid={r:.3e} fallbacks={fb}", flush=True)


if __name__ == "__main__":
    for (p, q) in [(2, 1), (2, 2)]:
        for la in (0, 2):
            for serial in ("0", "1"):
                run_dist(f, p * q, p, q, la, 1024, 128, serial, timeout=120)
