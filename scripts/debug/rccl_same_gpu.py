"""Probe: can two RCCL ranks share one GPU (for exercising the W=2 RCCL path on a 1-GPU
box)? Runs all_to_all_single with uneven splits + all_reduce; prints per-rank results."""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
W = dist.get_world_size()
send = [rank + 1 + p for p in range(W)]
recv = [p + 1 + rank for p in range(W)]
x = torch.full((sum(send), 4), float(rank), device="cuda")
y = torch.empty(sum(recv), 4, device="cuda")
dist.all_to_all_single(y, x, recv, send)
t = torch.ones(3, device="cuda") * (rank + 1)
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {rank}: a2a ok={bool((y[:recv[0]] == 0).all())} allreduce={t.tolist()}", flush=True)
dist.barrier()
dist.destroy_process_group()
