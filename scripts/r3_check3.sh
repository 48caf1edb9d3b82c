#!/usr/bin/env bash
# fused one-kernel layer: bitwise tests, full-scale check, step time with it on.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_f32_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "sage_fwd_fused or fused_fwd_bitwise" > gpurun_out/ffwd_tests.log 2>&1
rc=$?; tail -1 gpurun_out/ffwd_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/debug/ffwd_check.py > gpurun_out/ffwd_check.log 2>&1
rc=$?; grep -E "^(chunked|fused|h1 rows)" gpurun_out/ffwd_check.log; [ $rc -eq 0 ] || { tail -3 gpurun_out/ffwd_check.log; exit $rc; }
DGRAPH_FUSED_FWD=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extra > gpurun_out/ffwd_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/ffwd_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused-fwd step', d['ms_per_step'], d['final_loss'], json.dumps(d.get('regions',{}).get('ms_max_over_ranks')))"; exit $rc
