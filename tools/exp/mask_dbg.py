import sys, torch
sys.path.insert(0, '.')
from slate_amd import ops
def timeit(fn, reps=3):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
m = 16384
P = torch.randn(512, m, dtype=torch.float64, device='cuda').t(); C = torch.randn(m, m, dtype=torch.float64, device='cuda').t()
for name, mask in [("none", None), ("lower", (1, 1<<40, 1,0,1,0,0,0,0)), ("upper", (2, 1<<40, 1,0,1,0,0,0,0)),
                   ("skipall", (1, 1<<40, 1,0,1,0,0,0,-(1<<41))), ("lower_nb512", (1, 512, 1,0,1,0,0,0,0))]:
    print(name, f"{timeit(lambda: ops.gemm(-1.0, P, P, 1.0, C, 'N', 'T', mask)):.1f} us", flush=True)
