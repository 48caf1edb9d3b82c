#!/usr/bin/env bash
# Multi-process-on-one-GPU tests + native comm tests, then the fused fp32 papers100M step
# (timed) and its rocprofv3 kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_multiproc_gpu.py tests/test_comm_native_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/mp_tests.log 2>&1
echo "MP_RC=$?"; grep -E "PASS|FAIL|rel|Error" gpurun_out/mp_tests.log | grep -v "^E  *File" | tail -24
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extra > gpurun_out/fused_full.log 2>&1
echo "FULL_RC=$?"; grep '^{' gpurun_out/fused_full.log | cut -c1-300
TAG=fused TMO=400 BENCH_ARGS="--steps 1 --warmup 1 --no-extra" bash scripts/profile.sh > gpurun_out/prof_fused.txt 2>&1
echo "PROF_RC=$?"
ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_fused/stdout.log | grep -o '[0-9.]*$')
echo "ms_per_step=$ms"
python3 scripts/prof_window.py gpurun_out/prof_fused $ms 45 > gpurun_out/prof_fused_window.txt
head -48 gpurun_out/prof_fused_window.txt | cut -c1-180
python3 scripts/prof_summary.py gpurun_out/prof_fused 5 | tail -1
rm -f gpurun_out/prof_fused/run_kernel_trace.csv  # large; the window summary is kept
