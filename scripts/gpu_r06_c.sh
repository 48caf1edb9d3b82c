#!/bin/bash
# Structureless link-rate sweep, then the RGAT rank-1 W=8 rehearsal (layer-0 recompute).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
GRAPH=structureless RUNS="8:40 8:75 8:110 8:153 2:75 2:153" bash scripts/gpu_r06_sweep.sh
rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
O=gpurun_out/r06
timeout -k 10 900 python -u benchmarks/bench_rgcn.py --model rgat --rehearse-world 8 \
  --rehearse-rank 1 --link-gbps 153 --steps 3 --warmup 1 > $O/rgat_w8r1_g153.out 2> $O/rgat_w8r1_g153.err
rc=$?; echo "== rgat w8r1 rc=$rc"; tail -2 $O/rgat_w8r1_g153.out; [ $rc -ne 0 ] && grep -i "error" $O/rgat_w8r1_g153.err | tail -3
exit 0
