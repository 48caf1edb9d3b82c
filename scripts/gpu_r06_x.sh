#!/bin/bash
# Deferred weight gradients through per-parameter buffers: GPU tests, GraphCast W=1 and W=8
# ranks 0 / 3.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/gc
O=gpurun_out/r06/gc
timeout -k 10 300 python -u -m pytest tests/test_deferred_wgrad_gpu.py tests/test_graphcast_gpu.py -m gpu -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/x_tests.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -2 $O/x_tests.log
case $rc in 0) ;; *) grep -E "Error|assert" $O/x_tests.log | head -20; exit $rc;; esac
TAG=11 WTAG=bs5 bash scripts/gpu_r06_v.sh
