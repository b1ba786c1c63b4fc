"""Probe: can two ranks share one GPU over RCCL (for multi-rank rehearsal on a 1-GPU box)?"""
import os, torch, torch.distributed as dist
r = int(os.environ["RANK"]); w = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((4,), float(r + 1), device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
b = torch.arange(8, dtype=torch.float64, device="cuda") * (r == 0)
dist.broadcast(b, 0)
torch.cuda.synchronize()
print(f"rank {r}: allreduce {t.tolist()} bcast {b.tolist()[:3]}", flush=True)
dist.destroy_process_group()
