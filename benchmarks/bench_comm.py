#!/usr/bin/env python3
"""Communication micro-benchmarks (experiments/Benchmarks/TestNCCL.py, graph_utils.py).

* ``gather`` / ``scatter`` (G1 index API, with and without a precomputed cache) on the
  reference's all-to-all pattern: one vertex per rank, every rank holds one edge to every
  other rank's vertex, ``--message-size`` features per row; per-iteration HIP-event times
  (barrier between iterations) saved as ``{log_dir}/NCCL_{op}[_with_cache]_times_{rank}.npy``
  like the reference;
* ``halo``: the same pattern through :class:`HaloExchange` (G3);
* ``a2a``: raw all-to-all-v bandwidth sweep (bytes per peer), torch/RCCL vs the native
  C++ RCCL executor vs the one-sided symmetric-heap puts (``--impl torch,native,shmem``),
  reporting bus bandwidth per GPU;
* ``overlap``: an all-to-all-v concurrent with a row-group SpMM on another stream (the
  halo/interior overlap of parallel/dist_graph.py): each alone, both together, and each
  one's slowdown.

``--backend rocshmem`` runs the G1 gather/scatter through the one-sided engine (remote
get / pre-summed puts over the IPC symmetric heap; the reference's
experiments/Benchmarks/TestNVSHMEM.py:19-193), saving ``NVSHMEM_{op}_times_{rank}.npy`` as
the reference does. ``--pg-backend gloo`` lets several ranks share one GPU (the one-sided
paths need no RCCL communicator). CPU/gloo runs work too (``--device cpu``).
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
    ap.add_argument("--backend", default="nccl", choices=["nccl", "rocshmem", "nvshmem", "mpi"])
    ap.add_argument("--pg-backend", default=None,
                    help="process-group backend under the engine (gloo: ranks may share a GPU)")
    ap.add_argument("--overlap-rows", type=int, default=1 << 22,
                    help="rows of the synthetic CSR of the overlap probe (avg degree 29)")
    a = ap.parse_args()

    from dgraph_amd import Communicator
    from dgraph_amd.comm.alltoallv import AllToAllV
    from dgraph_amd.plan.legacy_cache import NCCLGatherCacheGenerator, NCCLScatterCacheGenerator

    kw = {"pg_backend": a.pg_backend} if a.pg_backend else {}
    comm = Communicator.init_process_group(a.backend, **kw)
    rank, W = comm.get_rank(), comm.get_world_size()
    if a.device == "cuda":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    dev = torch.device(a.device, torch.cuda.current_device()) if a.device == "cuda" else \
        torch.device("cpu")
    one_sided = a.backend in ("rocshmem", "nvshmem")
    prefix = {"nccl": "NCCL", "rocshmem": "NVSHMEM", "nvshmem": "NVSHMEM", "mpi": "MPI"}[a.backend]
    os.makedirs(a.log_dir, exist_ok=True)
    results = {}
    ops = a.ops.split(",")
    x, place, src = all2all_pattern(W, rank, a.message_size, dev)
    idx = src.unsqueeze(0).to(dev)
    m = torch.stack([place, src]).to(dev)
    if W > 1 and one_sided:
        # local form: this rank's edges (rank -> every other rank's single vertex)
        owners = torch.tensor([j for j in range(W) if j != rank], dtype=torch.long,
                              device=dev).unsqueeze(0)
        lidx = torch.zeros_like(owners)
        y = torch.randn(1, W - 1, a.message_size, device=dev)
        for op in ("gather", "scatter"):
            if op not in ops:
                continue
            fn = (lambda: comm.gather(x, lidx, owners)) if op == "gather" else \
                (lambda: comm.scatter(y, lidx, owners, 1))
            timed(fn, a.warmup, dev)
            t = timed(fn, a.iters, dev)
            name = f"{prefix}_{op}"
            np.save(os.path.join(a.log_dir, f"{name}_times_{rank}.npy"), t)
            results[name] = {"median_ms": float(np.median(t)),
                             "p99_ms": float(np.percentile(t, 99))}
    elif W > 1:
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
                name = f"{prefix}_{op}{'_with_cache' if use_cache else ''}"
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
        np.save(os.path.join(a.log_dir, f"{prefix}_halo_times_{rank}.npy"), t)
        results["halo"] = {"median_ms": float(np.median(t))}
    if "a2a" in ops:
        import dgraph_amd.comm.alltoallv as A

        for impl in a.impl.split(","):
            if impl in ("native", "shmem") and dev.type != "cuda":
                continue
            if impl == "shmem":
                os.environ.setdefault("DGRAPH_SYMHEAP_BYTES", str(max(
                    int(s_) for s_ in a.sizes.split(",")) * W * 2 + (64 << 20)))
                from dgraph_amd.comm.symheap import SymmetricHeap

                SymmetricHeap.DEFAULT_BYTES = int(os.environ["DGRAPH_SYMHEAP_BYTES"])
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
    if "overlap" in ops and dev.type == "cuda":
        results["overlap"] = overlap_probe(comm, W, dev, a)
    if rank == 0:
        print(json.dumps({"world_size": W, "device": str(dev), "backend": a.backend,
                          **results}), flush=True)
    from dgraph_amd.comm.alltoallv import close_shmem_heaps

    close_shmem_heaps()
    comm.destroy()


def overlap_probe(comm, W, dev, a):
    """All-to-all-v (64 MiB per peer, bf16) concurrent with a row-group SpMM (F=128 bf16
    over a random CSR, avg degree 29) on a second stream: each alone, together, slowdowns.
    Per-kernel times from events on each stream, median of 5."""
    from dgraph_amd.comm.alltoallv import AllToAllV
    from dgraph_amd.ops import kernels as K

    R = a.overlap_rows
    g = torch.Generator(device=dev).manual_seed(0)
    deg = torch.full((R,), 29, dtype=torch.long, device=dev)
    rowptr = torch.zeros(R + 1, dtype=torch.long, device=dev)
    torch.cumsum(deg, 0, out=rowptr[1:])
    col = torch.randint(0, R, (R * 29,), generator=g, device=dev, dtype=torch.int32)
    xs = torch.randn(R, 128, device=dev).to(torch.bfloat16)
    ys = torch.empty_like(xs)
    rows = (64 << 20) // (2 * 256)
    send = torch.randn(rows * W, 256, device=dev).to(torch.bfloat16)
    out = torch.empty_like(send)
    ex = AllToAllV([rows] * W, [rows] * W, comm.group)
    s_comm = torch.cuda.Stream(dev)

    def run(do_a2a, do_spmm):
        torch.cuda.synchronize()
        if W > 1:
            dist.barrier()
        ev = {k: torch.cuda.Event(enable_timing=True) for k in ("a0", "a1", "s0", "s1")}
        if do_a2a:
            with torch.cuda.stream(s_comm):
                ev["a0"].record(s_comm)
                ex(send, out=out)
                ev["a1"].record(s_comm)
        if do_spmm:
            ev["s0"].record()
            K.spmm(rowptr, col, xs, ys)
            ev["s1"].record()
        torch.cuda.synchronize()
        return (ev["a0"].elapsed_time(ev["a1"]) if do_a2a else 0.0,
                ev["s0"].elapsed_time(ev["s1"]) if do_spmm else 0.0)

    res = {k: [] for k in ("a2a_alone", "spmm_alone", "a2a_concurrent", "spmm_concurrent")}
    for it in range(6):
        a_ms, _ = run(True, False)
        _, s_ms = run(False, True)
        ca, cs = run(True, True)
        if it:
            res["a2a_alone"].append(a_ms)
            res["spmm_alone"].append(s_ms)
            res["a2a_concurrent"].append(ca)
            res["spmm_concurrent"].append(cs)
    med = {k: float(np.median(v)) for k, v in res.items()}
    med["a2a_slowdown"] = med["a2a_concurrent"] / max(med["a2a_alone"], 1e-9)
    med["spmm_slowdown"] = med["spmm_concurrent"] / max(med["spmm_alone"], 1e-9)
    med["bytes_per_peer"] = rows * 256 * 2
    return med


if __name__ == "__main__":
    main()
