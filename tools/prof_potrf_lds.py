"""Phase breakdown of one potrf_lds launch (in-kernel clock64 stamps):
shader clocks spent in load / update / diag / solve / half-update / writeback,
plus total clocks and wall time -> effective shader clock."""
import sys
import torch
sys.path.insert(0, '.')
from slate_amd import _native

H = _native.hip()
for n in (128, 256, 512):
    X = torch.randn(n, n, dtype=torch.float64, device='cuda')
    S = X @ X.T + n * torch.eye(n, dtype=torch.float64, device='cuda')
    A = torch.empty(n, n, dtype=torch.float64, device='cuda').t()
    info = torch.zeros(1, dtype=torch.int64, device='cuda')
    prof = torch.zeros(8, dtype=torch.int64, device='cuda')
    for it in range(3):
        A.copy_(S)
        H.potrf_lds_profile(n, A.data_ptr(), n, info.data_ptr(), prof.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    p = prof.tolist()
    wall_us = p[7] / 100.0
    ghz = p[6] / (wall_us * 1e3) if wall_us else 0
    names = ["load", "update", "diag", "solve", "half", "wb"]
    print(f"n={n}: wall {wall_us:.1f} us, {p[6]} clk ({ghz:.2f} GHz), info={int(info.item())}; " +
          ", ".join(f"{nm} {v / max(ghz, 1e-9) / 1e3:.1f}us" for nm, v in zip(names, p[:6])), flush=True)
    L = torch.tril(A)
    print("   resid", ((L @ L.T - S).abs().max() / S.abs().max()).item(), flush=True)
