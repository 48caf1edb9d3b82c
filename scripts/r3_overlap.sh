#!/usr/bin/env bash
# Co-residency probe of the fused executor's chunk pipeline (SpMM || MFMA GEMM).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/bench_overlap_f32.py --N 256 > gpurun_out/overlap_n256.log 2>&1
rc=$?; grep '^\[overlap' gpurun_out/overlap_n256.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/overlap_n256.log; exit $rc; }
timeout -k 10 300 python -u benchmarks/bench_overlap_f32.py --N 192 --tiles 256,128 --grids 0,1,2 > gpurun_out/overlap_n192.log 2>&1
rc=$?; grep '^\[overlap' gpurun_out/overlap_n192.log; exit $rc
