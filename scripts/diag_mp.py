#!/usr/bin/env python3
"""Diagnose W=2 (two processes, one GPU, shmem transport) vs W=1 differences of the fused
fp32 bench step: per-parameter relative gradient error, W=1 run-to-run and pipeline
on/off differences for scale."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ["DGRAPH_A2A_IMPL"] = "shmem"
os.environ.setdefault("DGRAPH_SYMHEAP_BYTES", str(1 << 30))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from conftest import run_ranks  # noqa: E402


def rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def body(rank, world, gf):
    import test_multiproc_gpu as T

    torch.cuda.set_device(0)
    args = T._args(dtype="fp32", global_frac=gf)
    refs = []
    if rank == 0:
        refs.append(T._run(0, 1, args, torch.float32))
        refs.append(T._run(0, 1, args, torch.float32))
        os.environ["DGRAPH_FUSED_PIPELINE"] = "0"
        refs.append(T._run(0, 1, args, torch.float32))
    dist.barrier()
    os.environ["DGRAPH_FUSED_PIPELINE"] = "1"
    got = T._run(rank, world, args, torch.float32)
    os.environ["DGRAPH_FUSED_PIPELINE"] = "0"
    got_np = T._run(rank, world, args, torch.float32)
    from dgraph_amd.comm.alltoallv import close_shmem_heaps

    close_shmem_heaps()
    if rank == 0:
        names = ["ws0", "wn0", "b0", "ws1", "wn1", "b1", "ws2", "wn2", "b2"]
        print(f"gf={gf} losses W1 {refs[0]['losses'].tolist()} W2 {got['losses'].tolist()}")
        for i, n in enumerate(names):
            r = refs[0]["grads"][i]
            print(f"{n:4s} |g|={float(r.norm()):.3e} W1rerun={rel(refs[1]['grads'][i], r):.2e} "
                  f"W1nopipe={rel(refs[2]['grads'][i], r):.2e} W2={rel(got['grads'][i], r):.2e} "
                  f"W2nopipe={rel(got_np['grads'][i], r):.2e} "
                  f"maxabs={float((got['grads'][i] - r).abs().max()):.2e}", flush=True)


if __name__ == "__main__":
    for gf in (0.05,):
        run_ranks(body, 2, gf, timeout=300)
