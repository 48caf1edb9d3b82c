#!/usr/bin/env python3
"""Per-parameter first-step gradient difference W=2 (two processes, one GPU, shmem
transport) vs W=1 of the bench step at a given hidden width (debug for the hidden-512
multi-process test)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
os.environ.setdefault("DGRAPH_A2A_IMPL", "shmem")
os.environ.setdefault("DGRAPH_SYMHEAP_BYTES", str(1 << 30))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from conftest import run_ranks  # noqa: E402


def body(rank, world, hidden):
    import test_multiproc_gpu as T

    torch.cuda.set_device(0)
    args = T._args(dtype="fp32", global_frac=0.05, hidden=hidden,
                   seed=int(os.environ.get("SEED", "0")))
    ref = T._run(0, 1, args, torch.float32, steps=1) if rank == 0 else None
    dist.barrier()
    got = T._run(rank, world, args, torch.float32, steps=1)
    from dgraph_amd.comm.alltoallv import close_shmem_heaps

    close_shmem_heaps()
    if rank == 0:
        names = [f"l{i}.{n}" for i in range(3) for n in ("w_self", "w_neigh", "bias")]
        print(f"hidden {hidden}: loss {float(got['losses'][0]):.8f} vs {float(ref['losses'][0]):.8f}",
              flush=True)
        for n, a, b in zip(names, got["grads"], ref["grads"]):
            rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
            print(f"  {n:12s} shape {tuple(a.shape)} rel {rel:.3e} max {float((a - b).abs().max()):.3e}",
                  flush=True)


if __name__ == "__main__":
    for h in [int(v) for v in sys.argv[1:]] or [512, 256]:
        run_ranks(body, 2, h, timeout=300)
