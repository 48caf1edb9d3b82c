#!/usr/bin/env bash
# Multi-process-on-one-GPU tests, native comm tests, GEMM probe, fused-step kernel profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_multiproc_gpu.py tests/test_comm_native_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/mp_tests.log 2>&1
echo "MP_RC=$?"; grep -E "PASS|FAIL|Error|error" gpurun_out/mp_tests.log | tail -20
timeout -k 10 200 python -u benchmarks/bench_fp32_probe.py --skip-spmm > gpurun_out/fp32_probe_gemm.log 2>&1
echo "PROBE_RC=$?"; grep -v '^{' gpurun_out/fp32_probe_gemm.log | grep -v amdgpu.ids | tail -16
TAG=fused TMO=500 BENCH_ARGS="--steps 1 --warmup 1 --no-extra" bash scripts/profile.sh > gpurun_out/prof_fused.txt 2>&1
echo "PROF_RC=$?"
ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_fused/stdout.log | grep -o '[0-9.]*$')
echo "ms_per_step=$ms"
python3 scripts/prof_window.py gpurun_out/prof_fused $ms 40 > gpurun_out/prof_fused_window.txt
head -45 gpurun_out/prof_fused_window.txt | cut -c1-200
