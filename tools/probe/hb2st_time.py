"""Time of the GPU bulge chase (hb2st.hip) alone vs the host pipeline, for
a random Hermitian band; argv: n b [workgroups...]."""
import os
import sys
import time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from slate_amd.models import eig as E

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
b = int(sys.argv[2]) if len(sys.argv) > 2 else 64
wgs = [int(x) for x in sys.argv[3:]] or [0]
g = torch.Generator().manual_seed(1)
X = torch.randn(n, n, generator=g, dtype=torch.float64)
H = X + X.T
i = torch.arange(n)
H = torch.where((i[:, None] - i[None, :]).abs() <= b, H, torch.zeros_like(H))
dev = torch.device("cuda")
os.environ["SLATE_AMD_HB2ST"] = "device"
for wg in wgs:
    if wg:
        os.environ["SLATE_AMD_HB2ST_WG"] = str(wg)
    E.hb2st(H, b, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d, e, F = E.hb2st(H, b, device=dev)
    torch.cuda.synchronize()
    print(f"device n={n} b={b} wg={wg or 'auto'}: {time.perf_counter() - t0:.3f} s", flush=True)
# per-phase clock totals (wait, reflector, left, right, finish) of one run
E._HB2ST_PROF["buf"] = torch.zeros(5, dtype=torch.int64, device=dev)
E.hb2st(H, b, device=dev)
torch.cuda.synchronize()
pv = E._HB2ST_PROF.pop("buf").cpu().tolist()
tot = max(sum(pv), 1)
print("phases (wait, reflector, left, right, finish):", ", ".join(f"{100 * x / tot:.1f}%" for x in pv),
      f"total {tot:.3e} cycles", flush=True)
if os.environ.get("HB2ST_PROBE_NOHOST"):
    sys.exit(0)
os.environ["SLATE_AMD_HB2ST"] = "host"
t0 = time.perf_counter()
d2, e2, F2 = E.hb2st(H, b, device=dev)
print(f"host   n={n} b={b}: {time.perf_counter() - t0:.3f} s", flush=True)
T1 = torch.diag(d) + torch.diag(e, 1) + torch.diag(e, -1)
T2 = torch.diag(d2) + torch.diag(e2, 1) + torch.diag(e2, -1)
print("eig diff", float((torch.linalg.eigvalsh(T1) - torch.linalg.eigvalsh(T2)).abs().max()), flush=True)
