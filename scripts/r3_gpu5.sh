#!/usr/bin/env bash
# fp32 kernel tests, GEMM/wgrad probe, headline bench with the persistent GEMM
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_f32_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1
rc=$?; echo "TESTS_RC=$rc"; tail -4 gpurun_out/f32_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/bench_fp32_probe.py --skip-spmm > gpurun_out/fp32_probe_gemm.log 2>&1 || { tail gpurun_out/fp32_probe_gemm.log; exit 1; }
grep '^\[' gpurun_out/fp32_probe_gemm.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extra > gpurun_out/fused_full.log 2>&1
echo "FULL_RC=$?"; grep '^{' gpurun_out/fused_full.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['peak_mem_gb_rank0'], json.dumps(d.get('regions',{}).get('ms_max_over_ranks')))"
