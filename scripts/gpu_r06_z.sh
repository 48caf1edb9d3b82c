#!/bin/bash
# Kernel trace of the final GraphCast W=8 rank 3 (eager), summarised per step on the box.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/gc
O=$R/gpurun_out/r06/gc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_gc -o prof -- \
  python3 $R/benchmarks/bench_graphcast.py --mode step --steps 5 --warmup 2 --partition aligned \
  --rehearse-world 8 --rehearse-rank 3 --link-gbps 153 > $O/prof_w8r3_final.log 2>&1
echo "== prof rc=$?"
DB=$(find /tmp/prof_gc -name "*.db" | head -1)
python3 $R/scripts/prof_db_steps.py "$DB" --total-steps 8 --steps 4 --skip-last 1 --top 60 \
  > $O/prof_w8r3_final_kernels_per_step.txt
head -45 $O/prof_w8r3_final_kernels_per_step.txt | cut -c1-170
rm -rf /tmp/prof_gc
