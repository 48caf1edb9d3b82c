#!/bin/bash
# GraphCast branch stream with event joins (mesh / m2m / m2g embeddings on the branch): GPU
# tests, W=1, W=8 ranks 0-3.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/gc
O=gpurun_out/r06/gc
timeout -k 10 300 python -u -m pytest tests/test_graphcast_gpu.py -m gpu -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/v_tests.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -2 $O/v_tests.log
case $rc in 0) ;; *) grep -E "Error|assert" $O/v_tests.log | head; exit $rc;; esac
timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --steps 20 --warmup 3 \
  --cuda-graph > $O/w1_${WTAG:-bs2}_graph.log 2>&1 || exit $?
grep '^{' $O/w1_${WTAG:-bs2}_graph.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('w1', round(d['ms_per_step'],2))"
RANKS="0 1 2 3" TAG=${TAG:-8} bash scripts/gpu_r06_k.sh
