#!/usr/bin/env bash
# col-map compaction: kernel tests, headline step (3 steps), products fp32 vs bf16.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_f32_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1
rc=$?; tail -2 gpurun_out/f32_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/f32_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extra > gpurun_out/cmap_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/cmap_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('step', d['ms_per_step'], d['final_loss'], json.dumps(d.get('regions',{}).get('ms_max_over_ranks')))"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --shape ogbn-products --steps 10 --warmup 2 --no-extra > gpurun_out/products_fp32.log 2>&1
rc=$?; grep '^{' gpurun_out/products_fp32.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('products fp32', d['ms_per_step'], d['executor'], d['value'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --shape ogbn-products --steps 10 --warmup 2 --no-extra --dtype bf16 --executor stack > gpurun_out/products_bf16.log 2>&1
rc=$?; grep '^{' gpurun_out/products_bf16.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('products bf16', d['ms_per_step'], d['executor'], d['value'])"; exit $rc
