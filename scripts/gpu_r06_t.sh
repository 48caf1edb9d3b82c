#!/bin/bash
# Deferred weight gradients assigned directly: GraphCast GPU tests, W=1 and W=8 rank 0 / 3.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/gc
O=gpurun_out/r06/gc
timeout -k 10 300 python -u -m pytest tests/test_graphcast_gpu.py tests/test_indexmap_hub_split.py -m gpu -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_tests.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -2 $O/t_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --steps 20 --warmup 3 \
  --cuda-graph > $O/w1_ws1b_graph.log 2>&1 || exit $?
grep '^{' $O/w1_ws1b_graph.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('w1', round(d['ms_per_step'],2))"
RANKS="0 3" TAG=6 bash scripts/gpu_r06_k.sh
