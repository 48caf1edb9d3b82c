"""Allocator probe of the 1-GPU papers100M step: per-step time, allocation retries
(cudaMalloc failures that made the caching allocator release blocks), reserved vs
allocated, device total. Usage: DGRAPH_BENCH_GRAD_SUPPORT=on python scripts/debug/alloc_probe.py"""
import argparse
import os
import sys
import time
import types

os.environ.setdefault("PYTORCH_ALLOC_CONF", "max_split_size_mb:512")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

a = argparse.Namespace(shape="ogbn-papers100M", scale=1.0, hidden=256, layers=3, lr=1e-3,
                       dtype="bf16", global_frac=0.05, window=1 << 14, seed=0, no_overlap=False,
                       rehearse_world=0, rehearse_rank=0, halo_recompute="off", cuda_graph=False)
comm = types.SimpleNamespace(get_rank=lambda: 0, get_world_size=lambda: 1, group=None)
dev = torch.device("cuda", 0)
print("device total GB", torch.cuda.get_device_properties(0).total_memory / 1e9, flush=True)
job = bench.Job(a, comm, dev, 0.05, torch.bfloat16)
for i in range(5):
    torch.cuda.synchronize()
    t = time.perf_counter()
    job.step(False)
    torch.cuda.synchronize()
    st = torch.cuda.memory_stats()
    print(f"step {i}: {1e3 * (time.perf_counter() - t):.1f} ms retries "
          f"{st.get('num_alloc_retries', 0)} allocated {st['allocated_bytes.all.current'] / 1e9:.1f} "
          f"reserved {st['reserved_bytes.all.current'] / 1e9:.1f} peak "
          f"{st['allocated_bytes.all.peak'] / 1e9:.1f} GB, free "
          f"{torch.cuda.mem_get_info()[0] / 1e9:.1f} GB", flush=True)
