"""Time the divide & conquer tridiagonal eigensolver (models/stedc.py) on
one GPU: n = 16384 random tridiagonal, leaves on the GPU, split merge GEMMs.
Prints the time of each of 3 runs and a residual / orthogonality sample."""
import sys
import time

import numpy as np
import torch

from slate_amd.models.stedc import stedc_rows

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
dev = torch.device("cuda")
rng = np.random.default_rng(0)
d, e = rng.standard_normal(n), rng.standard_normal(n - 1)
for it in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    w, Q, r0, r1, _ = stedc_rows(d, e, None, dev)
    torch.cuda.synchronize()
    print(f"stedc n={n} run {it}: {time.perf_counter() - t0:.3f} s", flush=True)
# residual on 256 random columns: T q - w q
cols = torch.from_numpy(rng.choice(n, 256, replace=False)).to(dev)
Qc = Q[:, cols]
dd, ee = torch.from_numpy(d).to(dev), torch.from_numpy(e).to(dev)
TQ = dd[:, None] * Qc
TQ[:-1] += ee[:, None] * Qc[1:]
TQ[1:] += ee[:, None] * Qc[:-1]
res = (TQ - Qc * w.to(dev)[cols]).abs().max().item()
orth = (Qc.T @ Qc - torch.eye(256, dtype=torch.float64, device=dev)).abs().max().item()
ref = np.linalg.eigvalsh(np.diag(d) + np.diag(e, 1) + np.diag(e, -1)) if n <= 4096 else None
print(f"residual {res:.2e} orthogonality {orth:.2e}" +
      (f" eig err {np.abs(w.numpy() - ref).max():.2e}" if ref is not None else ""), flush=True)
