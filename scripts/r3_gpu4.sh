#!/usr/bin/env bash
# fp32 kernel tests + fused-step bench (timed) + kernel-window profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_f32_kernels_gpu.py tests/test_alloc_steady_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1
echo "TESTS_RC=$?"; tail -4 gpurun_out/f32_tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extra > gpurun_out/fused_full.log 2>&1
echo "FULL_RC=$?"; grep '^{' gpurun_out/fused_full.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['peak_mem_gb_rank0'], json.dumps(d.get('regions',{}).get('ms_max_over_ranks')))"
TAG=fused TMO=400 BENCH_ARGS="--steps 1 --warmup 1 --no-extra" bash scripts/profile.sh > gpurun_out/prof_fused.txt 2>&1
echo "PROF_RC=$?"
ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_fused/stdout.log | grep -o '[0-9.]*$')
echo "ms_per_step=$ms"
python3 scripts/prof_window.py gpurun_out/prof_fused $ms 25 > gpurun_out/prof_fused_window.txt
head -27 gpurun_out/prof_fused_window.txt | cut -c1-170
rm -f gpurun_out/prof_fused/run_kernel_trace.csv
