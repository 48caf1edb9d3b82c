#!/usr/bin/env python3
"""One-sided symmetric-heap kernels on ONE GPU (csrc/comm/symheap.hip): the device cost of
the rocshmem/nvshmem transport with the link taken out.

A world-1 :class:`~dgraph_amd.comm.symheap.SymmetricHeap` maps its own heap as the only
peer, so ``heap_get_rows`` (the K15 remote get, the reference's ``dist_get``,
DGraph/distributed/csrc/torch_nvshmem_p2p.cu:166-235) and ``heap_put_rows`` (the put at
remote offsets) run their real kernels against local HBM: the achieved bytes per second are
the rate the kernels can feed, which the xGMI links (≈153 GB/s per peer, 7 peers) then
bound on a node. Also timed: the stream-ordered completion round trip (``heap_signal`` +
``heap_wait`` with ``self_too``), i.e. what one device-side barrier costs when no peer
lags — the reference benchmarked its NVSHMEM exchanges the same way (1000 iterations,
events, experiments/Benchmarks/TestNVSHMEM.py:28-88).

    python benchmarks/bench_heap.py [--rows 4194304] [--widths 64,128,256] [--iters 50]

One JSON line per measurement.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 22)
    ap.add_argument("--widths", default="64,128,256")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from dgraph_amd import _native
    from dgraph_amd.comm.symheap import _PUT, SymmetricHeap

    ops = _native.ops()
    dev = torch.device("cuda", 0)
    n = a.rows
    widths = [int(w) for w in a.widths.split(",")]
    fmax = max(widths)
    heap = SymmetricHeap(2 * n * fmax * 4 + (64 << 20), group=None, device=dev)
    src = heap.alloc_tensor((n, fmax), torch.float32)
    dst = heap.alloc_tensor((n, fmax), torch.float32)
    src.uniform_()
    g = torch.Generator(device=dev).manual_seed(0)
    owners = torch.zeros(n, dtype=torch.long, device=dev)
    for order in ("sequential", "random"):
        rows = torch.arange(n, device=dev) if order == "sequential" else \
            torch.randperm(n, device=dev, generator=g)
        for F in widths:
            x = src[:, :F]
            out = torch.empty(n, F, device=dev)
            nbytes = 2 * n * F * 4  # read + write

            def get():
                ops.heap_get_rows(heap.table, heap.offset_of(src), owners, rows, out,
                                  src.stride(0))

            ms = timed(get, a.iters)
            assert torch.equal(out, x[rows]), "heap_get_rows mismatch"
            ref_ms = timed(lambda: torch.index_select(x, 0, rows, out=out), a.iters)

            def put():
                ops.heap_put_rows(heap.table, heap.offset_of(dst), owners, rows,
                                  out, dst.stride(0))

            pms = timed(put, a.iters)
            print(json.dumps({"op": "heap_get_rows", "order": order, "rows": n, "F": F,
                              "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
                              "torch_index_select_GBps": round(nbytes / ref_ms / 1e6, 1)}),
                  flush=True)
            print(json.dumps({"op": "heap_put_rows", "order": order, "rows": n, "F": F,
                              "ms": round(pms, 4), "GBps": round(nbytes / pms / 1e6, 1)}),
                  flush=True)
    # completion round trip: signal (system-scope release store) + wait (acquire spin)
    ep = [0]

    def rt():
        ep[0] += 1
        heap.signal(_PUT, ep[0], self_too=True)
        heap.wait(_PUT, ep[0], self_too=True)

    us = timed(rt, 1000) * 1e3
    heap.check()
    print(json.dumps({"op": "signal_wait_round_trip", "us": round(us, 2),
                      "note": "device-side, self as the only peer (no link latency)"}),
          flush=True)
    heap.close()


if __name__ == "__main__":
    main()
