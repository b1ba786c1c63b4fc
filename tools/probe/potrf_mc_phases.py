"""Phase stamps of the multi-workgroup tile Cholesky (potrf_mc): per launch,
the workgroup-0 (critical) phases in microseconds from the launch's first
stamp (one launch per block step: WG 0 = update of A_kk, its Cholesky and
inverses; phases 0 start, 1 loads, 2 solves, 3 syrk, 4 factor start,
5 elimination done, 6 end)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slate_amd import _native

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
H = _native.hip()
g = torch.Generator(device=dev).manual_seed(1)
X = torch.rand(n, n, dtype=torch.float64, device=dev, generator=g)
S = (X @ X.T + n * torch.eye(n, dtype=torch.float64, device=dev)).T.contiguous().T
A = S.clone()
info = torch.zeros(1, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream().cuda_stream
prof = torch.zeros(17 * 512, dtype=torch.int64, device=dev)
for it in range(3):
    A.copy_(S)
    prof.zero_()
    H.potrf_mc_set_prof(prof.data_ptr() if it == 2 else 0)
    H.potrf_tile_variant(1, n, A.data_ptr(), A.stride(1), info.data_ptr(), st)
    torch.cuda.synchronize()
H.potrf_mc_set_prof(0)
p = prof[:16 * 512].view(16, 64, 8).cpu()
t00 = int(p[0, 0, 0])
for L in range(16):
    row = p[L, 0]
    if int(row[0]) == 0:
        continue
    nz = [int(x) for x in row if int(x) != 0]
    rel = [(x - nz[0]) / 100.0 for x in nz]          # 100 MHz ticks -> us
    nwg = int((p[L, :, 0] != 0).sum())
    last = max(int(x) for x in p[L].flatten() if int(x) != 0)
    print(f"launch {L:2d} wgs={nwg:2d} start={(nz[0] - t00) / 100:7.1f} "
          f"wg0 phases={['%.1f' % r for r in rel]} launch_span={(last - nz[0]) / 100:.1f} us", flush=True)
# step stamps of WG 0 of launch 1 (shader clocks, buffer tail): per wave, step start and
# end of its work before the barrier
L = 1
q = prof.cpu()[16 * 512:16 * 512 + 4 * 24 * 2].view(4, 24, 2)
base = int(q[0, 0, 0])
for st in range(12):
    row = []
    for w in range(4):
        s0, s1 = int(q[w, st, 0]) - base, int(q[w, st, 1]) - base
        row.append(f"w{w}:{s0:6d}+{s1 - s0:4d}")
    print(f"step {st:2d} " + " ".join(row))
