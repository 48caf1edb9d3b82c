#!/usr/bin/env bash
# dual GEMM timing + HBM traffic counters on SAGE combine shapes
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/bench_dual_gemm.py --rows ${ROWS:-33554432} --shapes ${SHAPES:-256:256:256,256:192:0,256:128:128} > gpurun_out/dg_time.log 2>&1
COUNTERS="FETCH_SIZE" TAG=dg TMO=200 bash scripts/pmc.sh python3 benchmarks/bench_dual_gemm.py --rows ${ROWS:-33554432} --shapes ${SHAPES:-256:256:256,256:192:0,256:128:128}
