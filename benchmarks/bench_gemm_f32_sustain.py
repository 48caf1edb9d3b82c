#!/usr/bin/env python3
"""fp32 MFMA GEMM rate in short bursts vs sustained back-to-back runs (is the matrix-core
rate clock-limited under sustained load?), against the library fp32 GEMM (hipBLASLt via
torch.mm) on the same shape.

    python benchmarks/bench_gemm_f32_sustain.py [--rows 1438388]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1438388)
    a = ap.parse_args()
    from dgraph_amd import _native
    from dgraph_amd.ops import f32 as F32

    _native.load()
    dev = torch.device("cuda", 0)
    M = a.rows
    A1 = torch.randn(M, 512, device=dev)
    B1 = torch.randn(512, 256, device=dev) / 22
    out = torch.empty(M, 256, device=dev)
    flops = 2 * M * 512 * 256
    res = {}

    def run(name, fn):
        fn()
        torch.cuda.synchronize()
        for n in (1, 10, 100):
            torch.cuda.synchronize()
            torch.cuda._sleep(50_000_000)  # idle ~ tens of ms: let the clock recover
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(n):
                fn()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / n
            res[f"{name}_x{n}"] = {"ms": round(ms, 3), "TFps": round(flops / ms / 1e9, 1)}
            print(name, n, res[f"{name}_x{n}"], flush=True)

    run("gemm_f32", lambda: F32.gemm_f32(A1, B1, out=out))
    run("torch_mm", lambda: torch.mm(A1, B1, out=out))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
