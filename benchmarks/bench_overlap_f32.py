#!/usr/bin/env python3
"""Co-residency probe for the fused fp32 executor's two-stream chunk pipeline.

models/sage_fused.py runs chunk c+1's aggregation (memory-bound fp32 SpMM) on one stream
while chunk c's MFMA dual GEMM runs on another. Whether the two actually overlap depends on
whether their workgroups can share a CU: the default GEMM block (512 threads, ~240 VGPRs,
2 waves/SIMD) fills every SIMD's register file, so the SpMM's waves cannot sit next to it.
This probe times, on a papers100M-shaped graph (scaled), one hidden layer's chunk loop:

  spmm      : the aggregation of every chunk alone
  gemm      : the dual GEMM of every chunk alone
  pipe      : both through the executor's _Pipe (two streams, double buffers)

for each (GEMM tile, SpMM grid cap) schedule:
  gemm_tile 256 : the default GEMM block; 128 : the lean one-wave-per-SIMD block
  spmm_grid 0   : one row group per wave (whole chunk in one grid); k*CUs : persistent cap

    python benchmarks/bench_overlap_f32.py [--scale 0.25] [--N 256] [--K 512]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, reps=3):
    ts = []
    for r in range(reps + 1):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        if r:
            ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.25)
    ap.add_argument("--F", type=int, default=256, help="aggregated width")
    ap.add_argument("--N", type=int, default=256, help="GEMM output width")
    ap.add_argument("--chunk", type=int, default=1 << 21)
    ap.add_argument("--tiles", default="256,128")
    ap.add_argument("--grids", default="0,1,2,3")
    ap.add_argument("--prios", default="0,1", help="side-stream priority variants (1 = high)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from dgraph_amd import _native
    from dgraph_amd.data.synthetic import SHAPES, build_partition
    from dgraph_amd.models.sage_fused import _Pipe, _ranges
    from dgraph_amd.ops import f32 as F32

    ops = _native.ops()
    shape = SHAPES["ogbn-papers100M"].scaled(a.scale)
    p = build_partition(shape, 0, 1, dev)
    csr = p["csr"]
    L = p["L"]
    inv = csr.inv_degree()
    F, N = a.F, a.N
    h = torch.randn(L, F, device=dev)
    ws = torch.randn(F, N, device=dev) * 0.05
    wn = torch.randn(F, N, device=dev) * 0.05
    b = torch.randn(N, device=dev)
    out = torch.empty(L, N, device=dev)
    chunks = _ranges(L, a.chunk)
    bufs = [torch.empty(a.chunk, F, device=dev) for _ in range(2)]
    pipes = {}
    for pr in [int(v) for v in a.prios.split(",")]:
        os.environ["DGRAPH_FUSED_SIDE_PRIO"] = str(pr)
        pipes[pr] = _Pipe(dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    items = list(range(len(chunks)))

    def produce(ci, k):
        r0, r1 = chunks[ci]
        o = bufs[k][:r1 - r0]
        F32.spmm_f32(csr.rowptr[r0:r1 + 1], csr.col, h, o, row_scale=inv[r0:r1])
        return o

    def consume(ci, agg, k):
        r0, r1 = chunks[ci]
        F32.gemm_f32(h[r0:r1], ws, agg, wn, bias=b, relu=True, out=out[r0:r1])

    def spmm_only():
        for ci in items:
            produce(ci, ci % 2)

    def gemm_only():
        for ci in items:
            consume(ci, bufs[ci % 2][:chunks[ci][1] - chunks[ci][0]], ci % 2)

    def piped(pr):
        pipes[pr].run(items, produce, consume)

    flops = 2.0 * L * (2 * F) * N
    res = {"L": L, "nnz": csr.nnz, "F": F, "N": N, "chunks": len(chunks), "cus": ncu}
    ref = None
    for tile in [int(t) for t in a.tiles.split(",")]:
        for gk in [int(g) for g in a.grids.split(",")]:
            grid = gk * ncu * (2 if gk else 0)  # 256-thread blocks: 2 per CU per unit
            ops.set_f32_sched(grid, tile)
            t_s = _time(spmm_only)
            t_g = _time(gemm_only)
            for pr in pipes:
                t_p = _time(lambda: piped(pr))
                if ref is None:
                    ref = out.clone()
                    err = 0.0
                else:
                    err = (out - ref).abs().max().item()
                key = f"tile{tile}_grid{gk}_prio{pr}"
                res[key] = {"spmm_ms": round(t_s, 2), "gemm_ms": round(t_g, 2),
                            "pipe_ms": round(t_p, 2), "sum_ms": round(t_s + t_g, 2),
                            "max_ms": round(max(t_s, t_g), 2),
                            "gemm_TFps": round(flops / t_g / 1e9, 1), "max_abs_vs_first": err}
                print(f"[overlap] {key}: spmm {t_s:.2f} ms  gemm {t_g:.2f} ms "
                      f"({flops / t_g / 1e9:.1f} TF/s)  pipe {t_p:.2f} ms  (sum "
                      f"{t_s + t_g:.2f}, max {max(t_s, t_g):.2f})  err {err:.1e}", flush=True)
    ops.set_f32_sched(0, 256)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
