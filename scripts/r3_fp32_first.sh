#!/usr/bin/env bash
# Round 3 first GPU contact of the fp32 path: kernel numerics, kernel probe, fused bench
# at a small scale, then the full papers100M fp32 step on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_f32_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1
echo "TESTS_RC=$?"; tail -15 gpurun_out/f32_tests.log
timeout -k 10 420 python -u benchmarks/bench_fp32_probe.py > gpurun_out/fp32_probe.log 2>&1
echo "PROBE_RC=$?"; grep -v '^{' gpurun_out/fp32_probe.log | tail -30
timeout -k 10 200 python -u bench.py --scale 0.01 --steps 5 --warmup 2 --no-extra > gpurun_out/fused_small.log 2>&1
echo "SMALL_RC=$?"; tail -3 gpurun_out/fused_small.log | cut -c1-600
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-extra > gpurun_out/fused_full.log 2>&1
echo "FULL_RC=$?"; tail -4 gpurun_out/fused_full.log | cut -c1-1500
