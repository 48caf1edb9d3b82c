#!/usr/bin/env bash
# Kernel trace of the headline step in both graph localities; per-kernel totals over the
# timed-step window only (scripts/prof_window.py). Output: gpurun_out/prof_{hl,sl}/
set -eu
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export PYTHONUNBUFFERED=1
for spec in "hl 0.05" "sl 1.0"; do
  set -- $spec
  TAG=$1 TMO=${TMO:-400} BENCH_ARGS="--steps 2 --warmup 1 --no-extra --global-frac $2 ${EXTRA:-}" \
    bash scripts/profile.sh > gpurun_out/prof_$1.txt 2>&1
  ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_$1/stdout.log | grep -o '[0-9.]*$')
  python3 scripts/prof_window.py gpurun_out/prof_$1 $(python3 -c "print(2*$ms)") 40 \
    > gpurun_out/prof_$1_window.txt
  head -3 gpurun_out/prof_$1_window.txt
done
