#!/bin/bash
# Kernel trace of the structureless W=2 rank (153 GB/s link model), summarised on the box.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
O=$R/gpurun_out/r06
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace -d /tmp/prof_sl2 -o prof -- \
  python3 $R/bench.py --rehearse-world 2 --global-frac 1.0 --link-gbps 153 --steps 3 --warmup 1 \
  --no-extra > $O/sl_w2_prof.out 2> $O/sl_w2_prof.err
echo "== prof rc=$?"
DB=$(find /tmp/prof_sl2 -name "*.db" | head -1)
python3 $R/scripts/prof_db_steps.py "$DB" --total-steps 5 --steps 3 --skip-last 1 --top 40 \
  > $O/sl_w2_kernels_per_step.txt
head -30 $O/sl_w2_kernels_per_step.txt | cut -c1-180
rm -rf /tmp/prof_sl2
