#!/usr/bin/env python3
"""Calibration probe for the fp32 (reference-precision) path on MI355X.

* library fp32 GEMM (torch.mm -> hipBLASLt/rocBLAS) at the GraphSAGE combine shapes
  [M, K] @ [K, N], M = 4M rows: TF/s and the epilogue cost (addmm + relu passes);
* the fp32 CSR SpMM at the papers100M shape (F = 128, 256) through the native kernels.

    python benchmarks/bench_fp32_probe.py [--spmm-scale 1.0]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, reps=5):
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
    ap.add_argument("--M", type=int, default=1 << 22)
    ap.add_argument("--spmm-scale", type=float, default=1.0)
    ap.add_argument("--feats", default="128,256")
    ap.add_argument("--skip-gemm", action="store_true")
    ap.add_argument("--skip-spmm", action="store_true")
    ap.add_argument("--global-frac", type=float, default=0.05,
                    help="SpMM graph: fraction of uniformly random edges (1.0 = structureless)")
    ap.add_argument("--passes", default="64,128,256",
                    help="row-group column-pass widths to time")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    res = {}
    if not a.skip_gemm:
        M = a.M
        for K_, N_ in ((128, 256), (256, 256), (512, 256), (256, 176), (256, 192), (256, 172)):
            x = torch.randn(M, K_, device=dev)
            w = torch.randn(K_, N_, device=dev)
            b = torch.randn(N_, device=dev)
            out = torch.empty(M, N_, device=dev)
            ms = _time(lambda: torch.mm(x, w, out=out))
            ms_e = _time(lambda: (torch.addmm(b, x, w, out=out), out.relu_()))
            tf = 2 * M * K_ * N_ / ms / 1e9
            res[f"mm_K{K_}_N{N_}"] = {"ms": round(ms, 3), "TFps": round(tf, 1),
                                      "addmm_relu_ms": round(ms_e, 3)}
            print(f"[gemm] M={M} K={K_} N={N_}: {ms:.3f} ms {tf:.1f} TF/s; addmm+relu "
                  f"{ms_e:.3f} ms", flush=True)
            if N_ != 172:
                from dgraph_amd.ops.f32 import gemm_f32

                # error vs an fp64 reference, in units of sum_k |a_k b_k| (the scale an
                # fp32 product chain's rounding error is proportional to)
                ref64 = torch.relu(torch.addmm(b.double(), x.double(), w.double()))
                scale = (x.abs().double() @ w.abs().double()).clamp_min(1e-30)
                err_lib = ((out_lib := torch.relu(torch.addmm(b, x, w))).double() - ref64
                           ).abs().div(scale).max().item()
                del out_lib
                if K_ >= 256:  # dual form: two K/2 operands, one fused kernel
                    h = K_ // 2
                    x1, x2 = x[:, :h].contiguous(), x[:, h:].contiguous()
                    ms_n = _time(lambda: gemm_f32(x1, w[:h], x2, w[h:], bias=b, relu=True,
                                                  out=out))
                else:
                    ms_n = _time(lambda: gemm_f32(x, w, bias=b, relu=True, out=out))
                err = (out.double() - ref64).abs().div(scale).max().item()
                tfn = 2 * M * K_ * N_ / ms_n / 1e9
                res[f"gemm_f32_K{K_}_N{N_}"] = {
                    "ms": round(ms_n, 3), "TFps": round(tfn, 1),
                    "max_err_rel_sumabs": err, "torch_mm_err_rel_sumabs": err_lib}
                print(f"[gemm_f32] dual+bias+relu K={K_} N={N_}: {ms_n:.3f} ms "
                      f"{tfn:.1f} TF/s (max err / sum|ab| {err:.2e}; torch.mm fp32 "
                      f"{err_lib:.2e})", flush=True)
                del ref64, scale
            del x, w, out
        # weight gradient x^T g over tall M
        x = torch.randn(M, 256, device=dev)
        g = torch.randn(M, 256, device=dev)
        ms = _time(lambda: torch.mm(x.t(), g))
        res["wgrad_256x256"] = {"ms": round(ms, 3), "TFps": round(2 * M * 256 * 256 / ms / 1e9, 1)}
        print(f"[gemm] wgrad x^T g M={M}: {ms:.3f} ms {2 * M * 65536 / ms / 1e9:.1f} TF/s",
              flush=True)
        from dgraph_amd.ops.dense import wgrad

        ms = _time(lambda: wgrad(x, g))
        res["wgrad_chunked_256x256"] = {"ms": round(ms, 3),
                                        "TFps": round(2 * M * 256 * 256 / ms / 1e9, 1)}
        print(f"[gemm] wgrad chunked M={M}: {ms:.3f} ms {2 * M * 65536 / ms / 1e9:.1f} TF/s",
              flush=True)
        from dgraph_amd.ops.f32 import WgradAcc

        acc = WgradAcc(256, 256, dev)

        def _wg():
            acc.reset()
            acc.add(x, g)
            return acc.result()

        ms = _time(_wg)
        err = (_wg() - torch.mm(x.t(), g)).abs().max().item()
        res["wgrad_f32_native_256x256"] = {"ms": round(ms, 3),
                                           "TFps": round(2 * M * 65536 / ms / 1e9, 1),
                                           "max_err": err}
        print(f"[gemm] wgrad_f32 native M={M}: {ms:.3f} ms {2 * M * 65536 / ms / 1e9:.1f} "
              f"TF/s (max err {err:.2e})", flush=True)
        del x, g
        torch.cuda.empty_cache()
    if not a.skip_spmm:
        from dgraph_amd.data.synthetic import SHAPES, build_partition
        from dgraph_amd.ops import kernels as K

        shape = SHAPES["ogbn-papers100M"]
        if a.spmm_scale != 1.0:
            shape = shape.scaled(a.spmm_scale)
        p = build_partition(shape, 0, 1, dev, global_frac=a.global_frac)
        csr = p["csr"]
        inv = csr.inv_degree()
        from dgraph_amd import _native

        ops = _native.ops()
        for F in [int(f) for f in a.feats.split(",")]:
            x = torch.randn(p["L"], F, device=dev)
            out = torch.empty_like(x)
            nbytes = csr.nnz * (F * 4 + 4) + p["L"] * F * 4
            variants = [("generic", 0, -1)] + [(f"rowgroup{w}", 1, int(w))
                                               for w in a.passes.split(",")]
            for name, rg, pc in variants:
                if pc > F:
                    continue
                ops.set_spmm_f32_config(rg, pc)
                ms = _time(lambda: K.spmm(csr.rowptr, csr.col, x, out, row_scale=inv), reps=3)
                res[f"spmm_f32_F{F}_{name}"] = {"ms": round(ms, 2),
                                                "TBps_eff": round(nbytes / ms / 1e9, 2)}
                print(f"[spmm] fp32 gf={a.global_frac} F={F} {name}: {ms:.2f} ms {nbytes / ms / 1e9:.2f} TB/s eff",
                      flush=True)
            ops.set_spmm_f32_config(1, 64)
            del x, out
            torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
