#!/bin/bash
# RGAT: 1/8-scale step with the layer-0 remake (kernel trace), rank-1 W=8 with an instant
# loopback (exposed exchange = difference to the 153 GB/s run).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
O=$R/gpurun_out/r06
timeout -k 10 900 python -u benchmarks/bench_rgcn.py --model rgat --rehearse-world 8 \
  --rehearse-rank 1 --steps 3 --warmup 1 > $O/rgat_w8r1_g0.out 2> $O/rgat_w8r1_g0.err
rc=$?; echo "== rgat w8r1 g0 rc=$rc"; tail -1 $O/rgat_w8r1_g0.out | cut -c1-300
case $rc in 124|134|137|139) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof_rgat_eighth -o prof -- \
  python3 $R/benchmarks/bench_rgcn.py --model rgat --scale 0.125 --steps 3 --warmup 1 \
  > $O/rgat_eighth_prof.out 2> $O/rgat_eighth_prof.err
echo "== prof rc=$?"; tail -1 $O/rgat_eighth_prof.out | cut -c1-300
