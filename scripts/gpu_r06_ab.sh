#!/bin/bash
# Kernel traces of the final structureless W=8 and W=2 ranks (153 GB/s link model).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
O=$R/gpurun_out/r06
cd /tmp && export TMPDIR=/tmp
for W in 8 2; do
  timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/prof_s$W -o prof -- \
    python3 $R/bench.py --rehearse-world $W --global-frac 1.0 --link-gbps 153 --steps 3 --warmup 1 \
    --no-extra > $O/sl_w${W}_final_prof.out 2> $O/sl_w${W}_final_prof.err
  rc=$?; echo "== W=$W prof rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
  DB=$(find /tmp/prof_s$W -name "*.db" | head -1)
  python3 $R/scripts/prof_db_steps.py "$DB" --total-steps 5 --steps 3 --skip-last 1 --top 30 \
    > $O/structureless_w${W}_rank_kernels_per_step_final.txt
  head -8 $O/structureless_w${W}_rank_kernels_per_step_final.txt | cut -c1-160
  rm -rf /tmp/prof_s$W
done
