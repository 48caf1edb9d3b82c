"""One-sided transport probe over a job's own halo plan (run as a separate child job).

``python -m dgraph_amd.comm.shmem_probe --plan PLAN.json [--width 64] [--iters 5]`` in each
of W processes (env ``RANK`` / ``WORLD_SIZE`` / ``LOCAL_RANK`` / ``MASTER_ADDR`` /
``MASTER_PORT``; one process per GPU, or every rank on one GPU with
``DGRAPH_RCCL_SHARED_GPU=1``). ``PLAN.json`` holds this rank's ``send_splits`` /
``recv_splits`` (the row counts of the job's halo all-to-all-v). Every rank fills its send
rows with seeded random fp32 values and exchanges them three ways:

* ``torch_pg``: ``dist.all_to_all_single`` on RCCL — the reference receive buffer;
* ``put_rows``: one-sided puts into the receivers' symmetric-heap slots
  (comm/symheap.py ``SymmetricHeap.put_rows`` through ``AllToAllV._shmem``, the
  ``DGRAPH_A2A_IMPL=shmem`` transport), completion device-side when the ranks hold
  distinct GPUs (``mode: device``) and host-side when they share one (``mode: host``);
* ``remote_gather``: the receiver reads the same rows straight out of the owners' heaps
  (``SymmetricHeap.remote_gather``, the reference's ``dist_get``,
  DGraph/distributed/csrc/torch_nvshmem_p2p.cu:166-235; its latency benchmark is
  experiments/Benchmarks/TestNVSHMEM.py:28-88).

For each transport: bitwise equality with the torch-PG buffer (reduced over ranks), the
exchange time (max over ranks, ``iters`` back-to-back calls between events), the largest
per-peer message over that time (min over ranks: the slowest link's rate), and whether a
device-side wait timed out. Rank 0 prints one ``SHMEM_PROBE {json}`` line.

bench.py runs this AFTER its headline job, as a child process per rank (the ranks never
replace themselves): a fault here costs the probe, never the headline line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

PREFIX = "SHMEM_PROBE "


def _reduce(vals, op, dev):
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    if dist.get_world_size() > 1:
        dist.all_reduce(t, op=op)
    return t.tolist()


def _timed(fn, iters: int, dev) -> float:
    """ms per call of ``fn`` over ``iters`` back-to-back calls after a barrier."""
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dist.barrier()
    if dev.type != "cuda":
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        return (time.perf_counter() - t0) * 1e3 / iters
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize(dev)
    return s.elapsed_time(e) / iters


def run(send_splits, recv_splits, width: int = 64, iters: int = 5) -> dict:
    """The probe on an initialised process group (every rank calls it). Returns the record
    (identical on every rank)."""
    from .alltoallv import AllToAllV
    from .groups import default_device

    rank, world = dist.get_rank(), dist.get_world_size()
    if dist.get_backend() == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    fault = os.environ.get("DGRAPH_SHMEM_PROBE_FAULT", "")
    if fault == f"abort{rank}":  # failure-path test hook: die like a faulting kernel would
        os.abort()
    ss, rs = [int(v) for v in send_splits], [int(v) for v in recv_splits]
    if len(ss) != world or len(rs) != world:
        raise ValueError(f"plan has {len(ss)} peers, world is {world}")
    n_send, n_recv = sum(ss), sum(rs)
    gen = torch.Generator(device="cpu").manual_seed(4321 + rank)
    send = torch.rand(n_send, width, generator=gen).to(dev)
    ref = torch.empty(n_recv, width, device=dev)
    rec: dict = {"width": width, "iters": iters, "world": world,
                 "rows_sent_max": int(_reduce([n_send], dist.ReduceOp.MAX, dev)[0]),
                 "rows_recv_max": int(_reduce([n_recv], dist.ReduceOp.MAX, dev)[0])}
    peer_bytes = max(max(ss, default=0), max(rs, default=0)) * width * 4

    def a2a_torch():
        dist.all_to_all_single(ref, send, output_split_sizes=rs, input_split_sizes=ss)

    a2a_torch()
    ms = _timed(a2a_torch, iters, dev)
    ms_max = _reduce([ms], dist.ReduceOp.MAX, dev)[0]
    gb = _reduce([peer_bytes / (ms * 1e6) if ms > 0 else 0.0], dist.ReduceOp.MIN, dev)[0]
    rec["torch_pg"] = {"exchange_ms_max": round(ms_max, 4),
                       "largest_peer_GBps_min_over_ranks": round(gb, 2)}
    if dev.type != "cuda":
        rec["shmem"] = "unavailable (no GPU: the symmetric heap is device memory)"
        return rec

    from .symheap import SymmetricHeap

    rmax, smax = rec["rows_recv_max"], rec["rows_sent_max"]
    need = (max(rmax, 1) + max(smax, 1)) * width * 4 + (4 << 20)
    SymmetricHeap.DEFAULT_BYTES = max(need, 16 << 20)
    # both heap memory kinds: coarse-grained hipMalloc (the default) and fine-grained device
    # memory (DGRAPH_SYMHEAP_FINE=1), whose cross-GPU coherence does not rest on kernel
    # boundaries — the first multi-GPU run shows which one the transport may rely on
    for fine in (False, True):
        sub = _heap_variant(rec if not fine else rec.setdefault("fine_grained", {}), fine,
                            send, ref, ss, rs, width, iters, dev, peer_bytes, world)
        if sub is not None:
            rec["fine_grained" if fine else "heap_error"] = sub
    return rec


def _heap_variant(rec, fine, send, ref, ss, rs, width, iters, dev, peer_bytes, world):
    """Probe put_rows / remote_gather on one heap kind into ``rec``; returns an error record
    when the heap cannot be created (on every rank alike: the creation is collective)."""
    from .alltoallv import AllToAllV, close_shmem_heaps, shmem_heap

    old = os.environ.get("DGRAPH_SYMHEAP_FINE")
    os.environ["DGRAPH_SYMHEAP_FINE"] = "1" if fine else "0"
    try:
        heap = shmem_heap(None, dev)
    except Exception as e:  # noqa: BLE001 - recorded; a heap kind the runtime refuses
        return {"error": repr(e)[:300]}
    finally:
        if old is None:
            os.environ.pop("DGRAPH_SYMHEAP_FINE", None)
        else:
            os.environ["DGRAPH_SYMHEAP_FINE"] = old
    rank = dist.get_rank()
    n_recv = sum(rs)
    rec["mode"] = "device" if heap.device_completion else "host"
    rec["heap_bytes"] = heap.nbytes
    rec["heap_memory"] = "fine-grained" if fine else "coarse-grained"
    plan = AllToAllV(ss, rs)
    out = torch.empty_like(ref)

    def probe(name, fn):
        err, eq, ms = "", 0, 0.0
        try:
            for _ in range(2):
                fn()
            torch.cuda.synchronize(dev)
            heap.check()
            eq = int(torch.equal(out, ref))
            ms = _timed(fn, iters, dev)
            heap.check()
        except Exception as e:  # noqa: BLE001 - recorded, reduced over ranks
            err = repr(e)[:300]
        timed_out = int("timed out" in err)
        v = _reduce([eq, ms, peer_bytes / (ms * 1e6) if ms > 0 else 0.0, int(bool(err)),
                     timed_out], dist.ReduceOp.MIN, dev)
        vmax = _reduce([ms, int(bool(err)), timed_out], dist.ReduceOp.MAX, dev)
        r = {"bitwise_equal_to_torch": bool(v[0] == 1 and vmax[1] == 0),
             "exchange_ms_max": round(vmax[0], 4),
             "largest_peer_GBps_min_over_ranks": round(v[2], 2),
             "timed_out": bool(vmax[2])}
        if vmax[1]:
            r["error_on_some_rank"] = True
        if err:
            r["error_rank%d" % rank] = err
        rec[name] = r
        out.zero_()

    def put():
        plan._shmem(send, out).wait()

    probe("put_rows", put)
    # remote_gather of the same rows: received row k from peer q is row
    # (q's send offset for me) + k of q's send buffer
    pre = torch.tensor([0] + ss[:-1], dtype=torch.long).cumsum(0).to(dev)
    theirs = torch.empty_like(pre)
    dist.all_to_all_single(theirs, pre)
    owners = torch.repeat_interleave(torch.arange(world, device=dev),
                                     torch.tensor(rs, device=dev), output_size=n_recv)
    first = torch.tensor([0] + rs[:-1], dtype=torch.long).cumsum(0).to(dev)
    idx = theirs[owners] + torch.arange(n_recv, device=dev) - first[owners]

    def get():
        out.copy_(heap.remote_gather(send, idx, owners))

    probe("remote_gather", get)
    torch.cuda.synchronize(dev)
    close_shmem_heaps()
    return None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--plan", required=True)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args(argv)
    with open(a.plan) as f:
        plan = json.load(f)
    from .groups import ensure_process_group

    ensure_process_group("nccl" if torch.cuda.is_available() else "gloo")
    rec = run(plan["send_splits"], plan["recv_splits"], a.width, a.iters)
    if dist.get_rank() == 0:
        print(PREFIX + json.dumps(rec), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
