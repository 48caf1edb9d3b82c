#!/usr/bin/env bash
# dual-GEMM kernels: numerics tests, then timing of both variants on the papers100M combine
# shapes (N:K1:K2 as called by the SAGE stack)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "dual_gemm" --timeout 120 --timeout-method thread > gpurun_out/dg_tests.log 2>&1
tail -2 gpurun_out/dg_tests.log
timeout -k 10 400 python -u benchmarks/bench_dual_gemm.py --rows ${ROWS:-111059956} --variants 1,2 --no-library \
  --shapes ${SHAPES:-256:128:128,256:256:256,192:256:0,256:192:0} > gpurun_out/dg_ab.log 2>&1
cat gpurun_out/dg_ab.log | grep -v '^{'
