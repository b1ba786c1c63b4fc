"""One torch (hipBLASLt) fp64 NT GEMM of the potrf update shape, for the
kernel name (macro tile / depth / MFMA config) in a rocprofv3 trace."""
import torch
for k in (512, 1024):
    a = torch.randn(24576, k, dtype=torch.float64, device='cuda')
    c = torch.randn(24576, 24576, dtype=torch.float64, device='cuda')
    for _ in range(2):
        torch.addmm(c, a, a.t(), beta=1.0, alpha=-1.0, out=c)
    torch.cuda.synchronize()
print("done", flush=True)
