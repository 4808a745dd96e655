"""Probe: RCCL all-reduce captured inside a hipGraph (torch.cuda.graph), 2 ranks.
Runs ranks on GPU (LOCAL_RANK % device_count) so it can be tried on a 1-GPU box."""
import os, sys, time, torch, torch.distributed as dist
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) % torch.cuda.device_count())
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
t = torch.full((225152,), float(rank + 1), device=dev)
dist.all_reduce(t); torch.cuda.synchronize()
print(rank, "eager ok", t[0].item(), flush=True)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
x = torch.full((225152,), float(rank + 1), device=dev)
with torch.cuda.graph(g, stream=s):
    x.mul_(2.0)
    dist.all_reduce(x)
torch.cuda.synchronize()
x.fill_(float(rank + 1)); g.replay(); torch.cuda.synchronize()
print(rank, "graph replay value", x[0].item(), "expected", 2.0 * sum(range(1, world + 1)), flush=True)
torch.cuda.synchronize(); dist.barrier()
t0 = time.perf_counter()
for _ in range(200): g.replay()
torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 200
print(rank, f"replay {dt*1e6:.1f} us (mul + 900KB allreduce)", flush=True)
dist.destroy_process_group()
