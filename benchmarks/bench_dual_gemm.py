#!/usr/bin/env python3
"""Fused MFMA dual GEMM (csrc/kernels/dual_gemm.hip) vs hipBLASLt mm + addmm + the
bias/ReLU/mask kernel, on SAGE layer-combine shapes. Reports ms and effective TB/s of the
fused kernel's compulsory traffic (A1 + A2 read, out write)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=5):
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
    ap.add_argument("--rows", type=int, default=1 << 25)
    ap.add_argument("--shapes", default="256:128:128,256:256:256,256:192:192,192:256:0")
    ap.add_argument("--variants", default="2",
                    help="dual-GEMM kernels to time: 1 = column-half (B^T in LDS), "
                         "2 = B-stationary (default)")
    ap.add_argument("--no-library", action="store_true")
    a = ap.parse_args()
    from dgraph_amd import _native
    from dgraph_amd.ops import kernels as K
    from dgraph_amd.ops.dense import dual_gemm, tile32_mask_words

    M = a.rows
    dev = torch.device("cuda")
    res = {}
    for spec in a.shapes.split(","):
        N, K1, K2 = (int(v) for v in spec.split(":"))
        A1 = torch.randn(M, K1, device=dev, dtype=torch.bfloat16)
        A2 = torch.randn(M, K2, device=dev, dtype=torch.bfloat16) if K2 else None
        B1 = torch.randn(K1, N, device=dev, dtype=torch.bfloat16) / K1 ** 0.5
        B2 = torch.randn(K2, N, device=dev, dtype=torch.bfloat16) / max(K2, 1) ** 0.5 if K2 else None
        bias = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        mo = torch.empty(tile32_mask_words(M, N), dtype=torch.int64, device=dev)
        B1t = B1.t().contiguous()
        B2t = B2.t().contiguous() if K2 else None
        relu = K2 > 0
        # K2 == 0 is the SAGE last-layer combine: out = A1 B1 + bias + out (cin in place)
        cin = out if not K2 else None
        fused_v = {}
        for v in (int(x) for x in a.variants.split(",")):
            _native.ops().set_dual_gemm_variant(v)
            fused_v[v] = timeit(lambda: dual_gemm(A1, B1t, A2, B2t, bias=bias, cin=cin,
                                                  out=out, relu=relu,
                                                  mask_out=mo if relu else None))
        _native.ops().set_dual_gemm_variant(-1)
        fused = min(fused_v.values())
        bits = torch.empty(K.mask_words(M * N), dtype=torch.int32, device=dev)

        def lib():
            if K2:
                torch.mm(A1, B1, out=out)
            else:
                out.addmm_(A1, B1)
            if K2:
                out.addmm_(A2, B2)
            if relu:
                K.bias_relu_pack(out, bias, bits, relu=True)
            else:
                out.add_(bias.to(out.dtype))

        ref_ms = float("nan") if a.no_library else timeit(lib)
        nbytes = (M * (K1 + K2) + M * N * (1 if K2 else 2)) * 2
        res[spec] = {"fused_ms": fused, "library_ms": ref_ms, "speedup": ref_ms / fused,
                     "fused_TBps": nbytes / fused / 1e9,
                     "by_variant": {v: {"ms": t, "TBps": nbytes / t / 1e9}
                                    for v, t in fused_v.items()}}
        per = " ".join(f"v{v} {t:.2f} ms ({nbytes / t / 1e9:.2f} TB/s)" for v, t in fused_v.items())
        print(f"N={N} K1={K1} K2={K2}: {per} | mm+addmm+epilogue {ref_ms:.2f} ms | "
              f"x{ref_ms / fused:.2f}", flush=True)
        del A1, A2, out, mo, bits
        torch.cuda.empty_cache()
    print(json.dumps({"rows": M, "results": res}))


if __name__ == "__main__":
    main()
