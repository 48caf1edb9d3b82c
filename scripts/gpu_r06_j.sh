#!/bin/bash
# Kernel trace of the structureless W=8 rank (153 GB/s link model), summarised on the box.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
O=$R/gpurun_out/r06
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace -d /tmp/prof_sl -o prof -- \
  python3 $R/bench.py --rehearse-world 8 --global-frac 1.0 --link-gbps 153 --steps 3 --warmup 1 \
  --no-extra > $O/sl_w8_prof.out 2> $O/sl_w8_prof.err
echo "== prof rc=$?"
DB=$(find /tmp/prof_sl -name "*.db" | head -1)
python3 $R/scripts/prof_db_steps.py "$DB" --total-steps 5 --steps 3 --skip-last 1 --top 40 \
  > $O/sl_w8_kernels_per_step.txt
head -30 $O/sl_w8_kernels_per_step.txt | cut -c1-160
rm -rf /tmp/prof_sl
