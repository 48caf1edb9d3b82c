#!/usr/bin/env bash
# act kernels + GraphCast step (fused linear+act), bf16x3 GEMM probe, co-residency probe
# with a high-priority matrix stream.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_act_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/act_tests.log 2>&1
rc=$?; tail -3 gpurun_out/act_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/act_tests.log | head; exit $rc; }
timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --profile-ops gpurun_out/gc_ops.txt > gpurun_out/gc_73.log 2>&1
rc=$?; grep '^{' gpurun_out/gc_73.log | cut -c1-300; [ $rc -eq 0 ] || { tail -5 gpurun_out/gc_73.log; exit $rc; }
timeout -k 10 300 python -u benchmarks/bench_fp32_probe.py --skip-spmm --gemm-modes 256,3 > gpurun_out/x3_probe.log 2>&1
rc=$?; grep '^\[' gpurun_out/x3_probe.log; [ $rc -eq 0 ] || { tail -8 gpurun_out/x3_probe.log; exit $rc; }
bash scripts/r3_overlap2.sh
