"""Probe: heev phase breakdown on one GPU (host spans of trace blocks, synchronised)."""
import os, sys, time, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import slate_amd as sl
from slate_amd.utils.trace import Trace

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda", 0)
A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, device=dev)
A.insertLocalTiles(device=0)
sl.generate_matrix(A, "rands", seed=7)
Z = sl.Matrix(n, n, nb=nb, device=dev)
Z.insertLocalTiles(device=0)
torch.cuda.synchronize()
Trace.on()
t0 = time.perf_counter()
w = sl.heev(A, None, Z, {sl.Option.InnerBlocking: nb})
torch.cuda.synchronize()
t = time.perf_counter() - t0
Trace.off()
tot = {}
for e in Trace.events():
    if e["nest"] <= 2:
        tot[e["name"]] = tot.get(e["name"], 0.0) + e["stop"] - e["start"]
print(f"heev n={n} nb={nb} dist={os.environ.get('SLATE_AMD_EIG_DIST', '0')}: {t:.3f} s", flush=True)
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:12]:
    print(f"  {k:24s} {v:8.3f} s", flush=True)
