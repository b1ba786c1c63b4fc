"""Per-phase host wall time of one heev (he2hb / hb2st / stedc / back-
transforms), from the trace spans.  python tools/heev_phases.py [n] [nb]"""
import os
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import slate_amd as sl  # noqa: E402
from slate_amd.utils.trace import Trace  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 256
band = int(sys.argv[3]) if len(sys.argv) > 3 else 0
dev = torch.device("cuda", 0)


def one():
    A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, device=dev)
    A.insertLocalTiles(device=dev)
    sl.generate_matrix(A, "rands", seed=1)
    Z = sl.Matrix(n, n, nb=nb, device=dev)
    Z.insertLocalTiles(device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sl.heev(A, None, Z, {sl.Option.InnerBlocking: band} if band else {})
    torch.cuda.synchronize()
    return time.perf_counter() - t0


one()                                   # warmup (kernels, workspaces)
Trace.on(device_timing=True)
t = one()
Trace.off()
agg = defaultdict(float)
for e in Trace.events():
    agg[(e["kind"] + (" " * 2 * e["nest"]), e["name"])] += e["stop"] - e["start"]
print(f"heev n={n} nb={nb} band={band or 'default'}: {t:.3f} s")
for (kind, name), v in sorted(agg.items(), key=lambda kv: (kv[0][0], -kv[1])):
    if v > 1e-3 * t:
        print(f"  {kind:8s} {name:30s} {v:8.3f} s")
