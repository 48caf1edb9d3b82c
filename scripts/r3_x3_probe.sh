#!/usr/bin/env bash
# bf16x3 split-product GEMM vs exact-f32 MFMA (time + error vs fp64); fp32 SpMM pass widths
# on the structureless graph.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/bench_fp32_probe.py --skip-spmm --gemm-modes 256,3 > gpurun_out/x3_probe.log 2>&1
rc=$?; grep '^\[' gpurun_out/x3_probe.log; [ $rc -eq 0 ] || { tail -8 gpurun_out/x3_probe.log; exit $rc; }
timeout -k 10 400 python -u benchmarks/bench_fp32_probe.py --skip-gemm --global-frac 1.0 --passes 64,128,256 > gpurun_out/spmm_sl_probe.log 2>&1
rc=$?; grep '^\[' gpurun_out/spmm_sl_probe.log; exit $rc
