#!/usr/bin/env bash
# rocprofv3 kernel trace of the fused fp32 step; last-step kernel window summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=fused TMO=400 BENCH_ARGS="--steps 1 --warmup 1 --no-extra" bash scripts/profile.sh > gpurun_out/prof_fused.txt 2>&1
echo "PROF_RC=$?"
ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_fused/stdout.log | grep -o '[0-9.]*$')
echo "ms_per_step=$ms"
python3 scripts/prof_window.py gpurun_out/prof_fused $ms 40 > gpurun_out/prof_fused_window.txt
head -42 gpurun_out/prof_fused_window.txt | cut -c1-200
rm -f gpurun_out/prof_fused/run_kernel_trace.csv
