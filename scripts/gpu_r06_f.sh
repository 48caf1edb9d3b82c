#!/bin/bash
# RGAT 1/8-scale step under a kernel trace, summarised on the box (the trace database is
# too large to bring back): per-step kernel totals of the timed steps.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
O=$R/gpurun_out/r06
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace -d /tmp/prof_rgat -o prof -- \
  python3 $R/benchmarks/bench_rgcn.py --model rgat --scale 0.125 --steps 3 --warmup 1 \
  > $O/rgat_eighth_prof.out 2> $O/rgat_eighth_prof.err
echo "== prof rc=$?"; tail -1 $O/rgat_eighth_prof.out | cut -c1-300
DB=$(ls /tmp/prof_rgat/*.db 2>/dev/null | head -1); [ -z "$DB" ] && DB=$(find /tmp/prof_rgat -name "*.db" | head -1)
python3 $R/scripts/prof_db_steps.py "$DB" --total-steps 4 --steps 3 --top 40 > $O/rgat_eighth_kernels_per_step.txt
echo "== summary rc=$?"; head -20 $O/rgat_eighth_kernels_per_step.txt | cut -c1-160
rm -rf /tmp/prof_rgat
