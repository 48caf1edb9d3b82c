#!/usr/bin/env bash
# Kernel trace of one rank of the W-way papers100M partition (loopback exchange), per-kernel
# totals over the timed steps only. Output: gpurun_out/prof_reh{W}/, prof_reh{W}_window.txt
set -eu
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export PYTHONUNBUFFERED=1
W=${W:-8}
TAG=reh$W TMO=${TMO:-400} BENCH_ARGS="--steps 3 --warmup 1 --no-extra --rehearse-world $W --rehearse-rank ${RANK_OF:-1} ${EXTRA:-}" \
  bash scripts/profile.sh > gpurun_out/prof_reh$W.txt 2>&1
ms=$(grep -o '"ms_per_step_compute_loopback": [0-9.]*' gpurun_out/prof_reh$W/stdout.log | grep -o '[0-9.]*$')
python3 scripts/prof_window.py gpurun_out/prof_reh$W $(python3 -c "print(3*$ms)") 40 \
  > gpurun_out/prof_reh${W}_window.txt
head -25 gpurun_out/prof_reh${W}_window.txt
