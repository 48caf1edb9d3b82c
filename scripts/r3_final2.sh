#!/usr/bin/env bash
# smoke (both paths), the fused-layer full-scale check, default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; grep "smoke ok" gpurun_out/smoke.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/smoke.log; exit $rc; }
timeout -k 10 400 python -u scripts/debug/ffwd_check.py > gpurun_out/ffwd_check.log 2>&1
rc=$?; grep -E "^(chunked|fused|h1 rows)" gpurun_out/ffwd_check.log; [ $rc -eq 0 ] || { tail -3 gpurun_out/ffwd_check.log; }
timeout -k 10 560 python -u bench.py > gpurun_out/bench_final.log 2>&1
rc=$?; grep '^{' gpurun_out/bench_final.log | cut -c1-3500; exit $rc
