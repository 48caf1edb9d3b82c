#!/usr/bin/env bash
# fp32 SpMM pass widths on the structureless graph, then the default bench (headline + extras).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u benchmarks/bench_fp32_probe.py --skip-gemm --global-frac 1.0 --passes 64,128,256 > gpurun_out/spmm_sl_probe.log 2>&1
rc=$?; grep '^\[' gpurun_out/spmm_sl_probe.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/spmm_sl_probe.log; exit $rc; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench1.log 2>&1
rc=$?; grep '^{' gpurun_out/bench1.log | cut -c1-2500; exit $rc
