#!/bin/bash
# copy_rows with 4 rows in flight per lane group: kernel tests, pack-shape rate, then the
# structureless / windowed W=8 rehearsals (153 GB/s) and the fp32 / link-delay / multiproc tests.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/copy
O=gpurun_out/r06/copy
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_cpu.py -q -k "copy_rows" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "== copy tests rc=$rc"; tail -2 $O/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u benchmarks/bench_copy_rows.py > $O/bench_copy_rows.jsonl 2> $O/bench_copy_rows.err
rc=$?; echo "== bench rc=$rc"; cat $O/bench_copy_rows.jsonl
case $rc in 0) ;; *) tail -5 $O/bench_copy_rows.err; exit $rc;; esac
EXTRA="--global-frac 1.0" TESTS=0 RUNS="8:153" bash scripts/rehearse_linkdelay.sh || exit $?
TESTS=1 RUNS="8:153" bash scripts/rehearse_linkdelay.sh
