"""Where do foreign (torch compute) kernels of the 2-rank heev/hetrf come
from?  Runs the census problem under torch.profiler with Python stacks and
prints the stack of every aten op that launched a non-slate kernel."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))


def _trap():
    """print the Python stack of every gather / scatter on a CUDA tensor"""
    import traceback
    for owner, name in ((torch, "gather"), (torch.Tensor, "gather"), (torch.Tensor, "scatter_"),
                        (torch, "scatter"), (torch.Tensor, "scatter"), (torch, "take_along_dim"),
                        (torch.Tensor, "take_along_dim"), (torch.Tensor, "index_put_")):
        fn = getattr(owner, name)

        def wrap(*a, _fn=fn, _name=name, **k):
            if any(isinstance(x, torch.Tensor) and x.is_cuda for x in a):
                print(f"TRAP {_name}:", "".join(traceback.format_stack(limit=7)[:-1]), flush=True)
            return _fn(*a, **k)
        setattr(owner, name, wrap)


def _run(rank, size):
    _trap()
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

    from torch.utils._python_dispatch import TorchDispatchMode
    import traceback

    class Spy(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            nm = str(func)
            if rank == 0 and ("gather" in nm or "index_copy" in nm or "scatter" in nm):
                print(f"SPY {nm}:\n" + "".join(traceback.format_stack(limit=9)[:-2]), flush=True)
            return func(*args, **(kwargs or {}))

    with Spy():
        hetrf()
    torch.cuda.synchronize()
    for name, fn in (("heev", heev), ("hetrf", hetrf)):
        fn()
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
            fn()
            torch.cuda.synchronize()
        if rank == 0:
            bad = ("add_", "maximum", "eq", "any", "max", "isnan", "where", "sub", "mul", "arange", "cumsum")
            for ev in prof.key_averages(group_by_stack_n=6):
                if ev.key.startswith("aten::") or "gloo" in ev.key or "c10d" in ev.key:
                    if getattr(ev, "self_device_time_total", getattr(ev, "self_cuda_time_total", 0)) > 0:
                        print(f"[{name}] {ev.key} x{ev.count}")
                        for fr in ev.stack:
                            print("      ", fr)


if __name__ == "__main__":
    from dist_util import run_dist
    run_dist(_run, 2, timeout=240)
