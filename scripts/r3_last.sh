#!/usr/bin/env bash
# GraphCast ERA5-37 step with the fused MLP layers; structureless W=8 rank: the fused
# executor must refuse it with MemoryError (planned), not run out of memory mid-step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --channel-config era5-37 > gpurun_out/gc_227.log 2>&1
rc=$?; grep '^{' gpurun_out/gc_227.log | cut -c1-250; [ $rc -eq 0 ] || { tail -3 gpurun_out/gc_227.log; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-extra --global-frac 1.0 --rehearse-world 8 --rehearse-rank 3 > gpurun_out/sl_w8.log 2>&1
echo "sl_w8 rc=$?"; grep -E "MemoryError|rehearsal|Traceback" gpurun_out/sl_w8.log | cut -c1-300 | tail -3
exit 0
