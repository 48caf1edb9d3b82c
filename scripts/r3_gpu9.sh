#!/usr/bin/env bash
# bf16x3 GEMM kernel: tests, probe (exact-f32 vs x3 kernel), fused step with x3 GEMMs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_f32_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/x3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/x3_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/x3_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u benchmarks/bench_fp32_probe.py --skip-spmm --gemm-modes 256,x3k > gpurun_out/x3k_probe.log 2>&1
rc=$?; grep '^\[gemm_f32' gpurun_out/x3k_probe.log; [ $rc -eq 0 ] || { tail -8 gpurun_out/x3k_probe.log; exit $rc; }
DGRAPH_GEMM_X3=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extra > gpurun_out/x3_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/x3_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('x3 step', d['ms_per_step'], d['final_loss'], json.dumps(d.get('regions',{}).get('ms_max_over_ranks')))"; exit $rc
