"""Foreign (non-slate_hip, non-copy) GPU kernels launched by heev / getrf."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import slate_amd as sl
sys.path.insert(0, os.path.join(sys.path[0], "tests"))
from test_kernel_census_gpu import _foreign, _kernels  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda", 0)
A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=256, device=dev)
A.insertLocalTiles(device=dev)
sl.generate_matrix(A, "rands", seed=5)
Z = sl.Matrix(n, n, nb=256, device=dev)
Z.insertLocalTiles(device=dev)
sl.heev(A, None, Z, {sl.Option.Target: sl.Target.Devices})      # warm-up
A2 = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=256, device=dev)
A2.insertLocalTiles(device=dev)
sl.generate_matrix(A2, "rands", seed=5)
names = _kernels(lambda: sl.heev(A2, None, Z, {sl.Option.Target: sl.Target.Devices}))
f = _foreign(names)
print("heev n=%d: %d kernel names, %d launches; foreign: %d names, %d launches" %
      (n, len(names), sum(names.values()), len(f), sum(f.values())))
for k, v in sorted(f.items(), key=lambda kv: -kv[1]):
    print(f"{v:6d}  {k[:160]}")
