#!/bin/bash
# GraphCast branch stream: GPU tests, W=1 and W=8 ranks 0 / 3 with and without it.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/gc
O=gpurun_out/r06/gc
timeout -k 10 300 python -u -m pytest tests/test_graphcast_gpu.py -m gpu -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/u_tests.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -2 $O/u_tests.log
case $rc in 0) ;; *) grep -E "Error|assert" $O/u_tests.log | head; exit $rc;; esac
for bs in 1 0; do
  timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --steps 20 --warmup 3 \
    --cuda-graph --branch-streams $bs > $O/w1_bs${bs}_graph.log 2>&1 || exit $?
  grep '^{' $O/w1_bs${bs}_graph.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('w1 bs$bs', round(d['ms_per_step'],2))"
done
RANKS="0 3" TAG=7 bash scripts/gpu_r06_k.sh || exit $?
RANKS="0 3" TAG=7bs0 EXTRA="--branch-streams 0" bash scripts/gpu_r06_k.sh
