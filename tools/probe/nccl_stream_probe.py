"""Which stream does a torch ProcessGroupNCCL (RCCL) collective run on?
One rank, world size 1: a synchronous all_reduce issued from a side stream,
between two elementwise kernels on that stream; the profiler reports the
stream of each device activity."""
import os
import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
s = torch.cuda.Stream()
t = torch.ones(1 << 20, device="cuda")
with torch.cuda.stream(s):
    dist.all_reduce(t)
    dist.broadcast(t, 0)
torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CUDA, ProfilerActivity.CPU]) as prof:
    with torch.cuda.stream(s):
        t.mul_(2)
        dist.all_reduce(t)
        dist.broadcast(t, 0)
        w = dist.all_reduce(t, async_op=True)
        w.wait()
        t.mul_(2)
    torch.cuda.synchronize()
print("side stream id", s.stream_id, "handle", hex(s.cuda_stream), "default", torch.cuda.current_stream().stream_id)
for e in prof.events():
    if str(e.device_type).endswith("CUDA"):
        print(f"{e.name[:70]:70s} stream={getattr(e, 'device_resource_id', None)}")
dist.destroy_process_group()
