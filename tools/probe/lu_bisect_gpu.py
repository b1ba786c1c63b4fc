"""Probe: distributed getrf, GPU vs CPU (host kernels) after k steps, 2 gloo ranks on one GPU."""
import os, sys, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import slate_amd as sl
from slate_amd.core.enums import Option
from dist_util import run_dist


def f(rank, size, p, q, la, n, nb, serial, trials):
    os.environ["SLATE_AMD_SERIAL"] = serial
    torch.cuda.set_device(0)
    from slate_amd.models.aux import allgather_dense as D
    for trial in range(trials):
        for k in range(1, n // nb + 1):
            os.environ["SLATE_AMD_DEBUG_LU_STEPS"] = str(k)
            res = []
            for dev in ("cuda", "cpu"):
                A = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev)
                A.insertLocalTiles(device=0 if dev == "cuda" else -1)
                sl.generate_matrix(A, "rands", 4)
                piv = sl.Pivots()
                sl.getrf(A, piv, {Option.Lookahead: la})
                res.append((D(A).cpu(), piv.ipiv.clone()))
                if dev == "cuda":
                    import torch.distributed as dist
                    allp = [torch.zeros_like(piv.ipiv) for _ in range(size)]
                    dist.all_gather(allp, piv.ipiv.clone())
                    for r in range(1, size):
                        dd = (allp[r] != allp[0]).nonzero().flatten().tolist()
                        if dd and rank == 0:
                            print(f"  step {k}: rank {r} pivots differ from rank 0 at {dd[:8]}: "
                                  f"{allp[0][dd[:4]].tolist()} vs {allp[r][dd[:4]].tolist()}", flush=True)
            d = (res[0][0] - res[1][0]).abs()
            pd = (res[0][1] != res[1][1]).nonzero().flatten().tolist()
            if d.max() > 1e-10 or pd:
                bad = (d > 1e-10).nonzero()
                rows = sorted(set(bad[:, 0].tolist()))
                cols = sorted(set(bad[:, 1].tolist()))
                if rank == 0:
                    print(f"trial {trial} grid {p}x{q} la={la} serial={serial}: first diff after step {k}: "
                          f"max {d.max():.3e} rows {rows[:12]}..({len(rows)}) cols {cols[:6]}..{cols[-3:]}({len(cols)}) "
                          f"piv diff {pd[:10]}", flush=True)
                break
        else:
            if rank == 0:
                print(f"trial {trial} grid {p}x{q} la={la} serial={serial}: identical", flush=True)


if __name__ == "__main__":
    run_dist(f, 2, 2, 1, 0, 1024, 128, "1", 4, timeout=300)
    os.environ["SLATE_AMD_LU_PERSIST"] = "0"
    run_dist(f, 2, 2, 1, 0, 1024, 128, "1", 4, timeout=300)
