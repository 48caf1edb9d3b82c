#!/usr/bin/env python3
"""Communication micro-benchmarks (experiments/Benchmarks/TestNCCL.py, graph_utils.py).

* ``gather`` / ``scatter`` (G1 index API, with and without a precomputed cache) on the
  reference's all-to-all pattern: one vertex per rank, every rank holds one edge to every
  other rank's vertex, ``--message-size`` features per row; per-iteration HIP-event times
  (barrier between iterations) saved as ``{log_dir}/NCCL_{op}[_with_cache]_times_{rank}.npy``
  like the reference;
* ``halo``: the same pattern through :class:`HaloExchange` (G3);
* ``a2a``: raw all-to-all-v bandwidth sweep (bytes per peer), torch/RCCL vs the native
  C++ RCCL executor (``--impl``), reporting bus bandwidth per GPU.

CPU/gloo runs work too (``--device cpu``).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def all2all_pattern(W: int, rank: int, F: int, device):
    """Reference benchmark graph: edges (i -> j) for all i != j, placed on rank i."""
    place = torch.repeat_interleave(torch.arange(W), W - 1)
    src = torch.tensor([j for i in range(W) for j in range(W) if i != j], dtype=torch.long)
    x = torch.randn(1, 1, F, generator=torch.Generator().manual_seed(rank)).to(device)
    return x, place, src


def timed(fn, iters: int, device, barrier=True):
    times = np.zeros(iters)
    for i in range(iters):
        if device.type == "cuda":
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            times[i] = s.elapsed_time(e)
        else:
            import time

            t = time.perf_counter()
            fn()
            times[i] = (time.perf_counter() - t) * 1e3
        if barrier and dist.get_world_size() > 1:
            dist.barrier()
    return times


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="gather,scatter,halo,a2a")
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--message-size", type=int, default=128)
    ap.add_argument("--sizes", default="4096,65536,1048576,16777216,67108864")
    ap.add_argument("--impl", default="torch,native")
    ap.add_argument("--log-dir", default="logs")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args()

    from dgraph_amd import Communicator
    from dgraph_amd.comm.alltoallv import AllToAllV
    from dgraph_amd.plan.legacy_cache import NCCLGatherCacheGenerator, NCCLScatterCacheGenerator

    comm = Communicator.init_process_group("nccl")
    rank, W = comm.get_rank(), comm.get_world_size()
    dev = torch.device(a.device, torch.cuda.current_device()) if a.device == "cuda" else \
        torch.device("cpu")
    os.makedirs(a.log_dir, exist_ok=True)
    results = {}
    ops = a.ops.split(",")
    x, place, src = all2all_pattern(W, rank, a.message_size, dev)
    idx = src.unsqueeze(0).to(dev)
    m = torch.stack([place, src]).to(dev)
    if W > 1:
        for op in ("gather", "scatter"):
            if op not in ops:
                continue
            for use_cache in (False, True):
                if op == "gather":
                    cache = NCCLGatherCacheGenerator(src, place, src, 1, rank, W) if use_cache else None
                    fn = (lambda c=cache: comm.gather(x, idx, m, cache=c))
                else:
                    y = torch.randn(1, W - 1, a.message_size, device=dev)
                    cache = NCCLScatterCacheGenerator(src, place, src, 1, rank, W) if use_cache else None
                    fn = ((lambda c=cache: comm.scatter(y, cache=c)) if use_cache
                          else (lambda: comm.scatter(y, idx, m, 1)))
                timed(fn, a.warmup, dev)
                t = timed(fn, a.iters, dev)
                name = f"NCCL_{op}{'_with_cache' if use_cache else ''}"
                np.save(os.path.join(a.log_dir, f"{name}_times_{rank}.npy"), t)
                results[name] = {"median_ms": float(np.median(t)), "p99_ms": float(np.percentile(t, 99))}
    if "halo" in ops and W > 1:
        from dgraph_amd.parallel.halo import HaloExchange
        from dgraph_amd.plan.pattern import build_communication_pattern

        el = torch.stack([place, src], 1)
        cp = build_communication_pattern(el, torch.arange(W), rank, W, group=comm.group).to(dev)
        hx = HaloExchange(comm)
        xl = x[0]
        timed(lambda: hx(xl, cp), a.warmup, dev)
        t = timed(lambda: hx(xl, cp), a.iters, dev)
        np.save(os.path.join(a.log_dir, f"NCCL_halo_times_{rank}.npy"), t)
        results["halo"] = {"median_ms": float(np.median(t))}
    if "a2a" in ops:
        import dgraph_amd.comm.alltoallv as A

        for impl in a.impl.split(","):
            if impl == "native" and dev.type != "cuda":
                continue
            A.A2A_IMPL = impl
            for nbytes in (int(s) for s in a.sizes.split(",")):
                rows = max(nbytes // (2 * 256), 1)  # bf16 rows of 256 features
                send = torch.randn(rows * W, 256, device=dev).to(torch.bfloat16 if dev.type == "cuda" else torch.float32)
                ex = AllToAllV([rows] * W, [rows] * W, comm.group)
                out = torch.empty_like(send)
                n_it = max(5, min(a.iters, 200))
                timed(lambda: ex(send, out=out), 3, dev, barrier=False)
                t = timed(lambda: ex(send, out=out), n_it, dev, barrier=False)
                ms = float(np.median(t))
                peer_bytes = rows * 256 * send.element_size()
                busbw = peer_bytes * (W - 1) / (ms / 1e3) / 1e9 if W > 1 else 0.0
                results[f"a2a_{impl}_{peer_bytes}B"] = {"median_ms": ms, "busbw_GBps": busbw}
    if rank == 0:
        print(json.dumps({"world_size": W, "device": str(dev), **results}), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
