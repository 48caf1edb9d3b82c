#!/bin/bash
# Heap get/put with 4 rows in flight: native comm GPU tests (+ multi-device tests, skipped on
# one GPU), the heap rates, and the shared-GPU W=2 bench with the one-sided probe.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/heap
O=gpurun_out/r06/heap
timeout -k 10 500 python -u -m pytest tests/test_comm_native_gpu.py tests/test_multidevice_gpu.py \
  tests/test_graphcast_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/tests.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -3 $O/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u benchmarks/bench_heap.py > $O/bench_heap.jsonl 2> $O/bench_heap.err
rc=$?; echo "== bench_heap rc=$rc"; cat $O/bench_heap.jsonl | cut -c1-300
