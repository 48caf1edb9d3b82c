#!/bin/bash
# Hub-split transposed segment sums: GPU tests, GraphCast W=1 (graph replay), W=8 aligned
# ranks 0 / 1 / 3.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/gc
O=gpurun_out/r06/gc
timeout -k 10 400 python -u -m pytest tests/test_indexmap_hub_split.py tests/test_graphcast.py tests/test_graphcast_gpu.py -m gpu -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/hub_tests.log 2>&1
rc=$?; echo "== pytest rc=$rc"; tail -3 $O/hub_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --steps 20 --warmup 3 \
  --cuda-graph > $O/w1_hub_graph.log 2>&1 || exit $?
grep '^{' $O/w1_hub_graph.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('w1', round(d['ms_per_step'],2))"
RANKS="0 1 3" TAG=4 bash scripts/gpu_r06_k.sh
