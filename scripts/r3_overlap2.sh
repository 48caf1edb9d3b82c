#!/usr/bin/env bash
# Co-residency probe with a high-priority matrix stream (lean GEMM tile).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/bench_overlap_f32.py --N 256 --tiles 256,128 --grids 0 --prios 0,1 > gpurun_out/overlap2_n256.log 2>&1
rc=$?; grep '^\[overlap' gpurun_out/overlap2_n256.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/overlap2_n256.log; exit $rc; }
timeout -k 10 300 python -u benchmarks/bench_overlap_f32.py --N 192 --tiles 256,128 --grids 0 --prios 0,1 > gpurun_out/overlap2_n192.log 2>&1
rc=$?; grep '^\[overlap' gpurun_out/overlap2_n192.log; exit $rc
