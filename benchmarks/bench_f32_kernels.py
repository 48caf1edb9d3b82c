#!/usr/bin/env python3
"""The fp32 hot kernels of the headline step, each alone at its step shape, for counter
passes (rocprofv3 --pmc) and per-kernel timing:

* spmm_f32_rowgroup (64-column passes) over the papers100M-shaped CSR at F = 128 and 256;
* the column-mapped (CMAP) transposed aggregation of a gradient stored on ~30 % of rows;
* gemm_f32 dual GEMM K = 256 + 256, N = 256 (hidden layer) and N = 176 (output layer);
* wgrad_f32 [K = 256, N = 256] over a row chunk.

    python benchmarks/bench_f32_kernels.py [--scale 0.25] [--rows 1438388] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.25)
    ap.add_argument("--rows", type=int, default=1438388)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--global-frac", type=float, default=0.05)
    ap.add_argument("--window", type=int, default=1 << 14)
    ap.add_argument("--xcd", default="1", help="SpMM XCD-contiguous block remap: 0, 1 or "
                    "0,1 (A/B in one process)")
    ap.add_argument("--pass-cols", default="64", help="SpMM pass widths, comma-separated")
    ap.add_argument("--spmm-only", action="store_true")
    a = ap.parse_args()
    from dgraph_amd import _native
    from dgraph_amd.data.synthetic import SHAPES, build_partition
    from dgraph_amd.ops import f32 as F32

    _native.load()
    dev = torch.device("cuda", 0)
    shape = SHAPES["ogbn-papers100M"].scaled(a.scale)
    p = build_partition(shape, 0, 1, dev, global_frac=a.global_frac, window=a.window)
    csr = p["csr"]
    L = p["L"]
    inv = csr.inv_degree()
    res = {"nnz": csr.nnz, "rows": L}

    def timed(name, fn, nbytes=None, flops=None):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3 / a.reps
        r = {"ms": round(ms, 3)}
        if nbytes:
            r["TBps_eff"] = round(nbytes / ms / 1e9, 2)
        if flops:
            r["TFps"] = round(flops / ms / 1e9, 1)
        res[name] = r
        print(name, r, flush=True)

    g = torch.Generator(device=dev).manual_seed(0)
    S = torch.nonzero(torch.rand(L, generator=g, device=dev) < 0.3).reshape(-1)
    smap = torch.full((L,), -1, dtype=torch.int32, device=dev)
    smap[S] = torch.arange(S.numel(), dtype=torch.int32, device=dev)
    for xcd in [int(v) for v in a.xcd.split(",")]:
        _native.ops().set_f32_sched(-1, -1, xcd)
        sfx = f"_xcd{xcd}"
        for pcs in a.pass_cols.split(","):
            pc = int(pcs)
            for F in (128, 256):
                x = torch.randn(L, F, device=dev)
                out = torch.empty(L, F, device=dev)
                timed(f"spmm_f32_F{F}_pc{pc}{sfx}",
                      lambda: F32.spmm_f32(csr.rowptr, csr.col, x, out, row_scale=inv,
                                           pass_cols=pc),
                      nbytes=csr.nnz * (F * 4 + 4) + L * F * 4)
                del x, out
        # column-mapped: u stored on ~30 % of the rows
        u = torch.randn(S.numel(), 256, device=dev)
        out = torch.empty(L, 256, device=dev)
        for pc in (64, 128, 256):
            timed(f"spmm_f32_cmap_F256_pc{pc}{sfx}", lambda pc=pc: F32.spmm_f32(
                csr.rowptr, csr.col, u, out, col_map=smap, pass_cols=pc))
        del u, out
    _native.ops().set_f32_sched(-1, -1, 0)
    if a.spmm_only:
        print(json.dumps(res))
        return
    M = a.rows
    A1 = torch.randn(M, 256, device=dev)
    A2 = torch.randn(M, 256, device=dev)
    for N in (256, 176):
        B1 = torch.randn(256, N, device=dev) / 16
        B2 = torch.randn(256, N, device=dev) / 16
        bias = torch.randn(N, device=dev)
        o = torch.empty(M, N, device=dev)
        timed(f"gemm_f32_K512_N{N}", lambda: F32.gemm_f32(A1, B1, A2, B2, bias=bias,
                                                          relu=N == 256, out=o),
              flops=2 * M * 512 * N)
    G = torch.randn(M, 256, device=dev)
    acc = F32.WgradAcc(256, 256, dev)

    def wg():
        acc.reset()
        acc.add(A1, G)
        acc.result()

    timed("wgrad_f32_256x256", wg, flops=2 * M * 256 * 256)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
