"""Where do foreign (torch compute) kernels of the 2-rank heev/hetrf come
from?  Runs the census problem under torch.profiler with Python stacks and
prints the stack of every aten op that launched a non-slate kernel."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))


def _run(rank, size):
    import slate_amd as sl
    from torch.profiler import ProfilerActivity, profile
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    n, nb = 384, 64

    def heev():
        H = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=2, q=1, device=dev)
        H.insertLocalTiles(device=0)
        sl.generate_matrix(H, "rands", 6)
        Z = sl.Matrix(n, n, nb=nb, p=2, q=1, device=dev)
        Z.insertLocalTiles(device=0)
        sl.heev(H, None, Z)

    def hetrf():
        A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=2, q=1, device=dev)
        A.insertLocalTiles(device=0)
        sl.generate_matrix(A, "rands", 8)
        sl.hetrf(A, sl.Pivots())

    for name, fn in (("heev", heev), ("hetrf", hetrf)):
        fn()
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
            fn()
            torch.cuda.synchronize()
        if rank == 0:
            bad = ("add_", "maximum", "eq", "any", "max", "isnan", "where", "sub", "mul", "arange", "cumsum")
            for ev in prof.key_averages(group_by_stack_n=6):
                if ev.key.startswith("aten::") and any(ev.key.endswith(b) or ev.key == "aten::" + b for b in bad):
                    if getattr(ev, "device_time_total", getattr(ev, "cuda_time_total", 0)) > 0:
                        print(f"[{name}] {ev.key} x{ev.count}")
                        for fr in ev.stack:
                            print("      ", fr)


if __name__ == "__main__":
    from dist_util import run_dist
    run_dist(_run, 2, timeout=240)
