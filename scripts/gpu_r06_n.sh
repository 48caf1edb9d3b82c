#!/bin/bash
# Side-stream weight gradients + refit GraphCast weights: GPU test, W=1 A/B, W=8 aligned
# ranks 0-3 (4-7 mirror them) with the side stream and rank 3 without, then a kernel trace
# of rank 3 (eager), summarised per step on the box.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/gc
O=$R/gpurun_out/r06/gc
timeout -k 10 300 python -u -m pytest tests/test_graphcast_gpu.py -m gpu -q -k deferred \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/defer_tests.log 2>&1
rc=$?; echo "== pytest rc=$rc"; tail -3 $O/defer_tests.log
case $rc in 0) ;; *) exit $rc;; esac
for ws in 1 0; do
  timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --steps 20 --warmup 3 \
    --cuda-graph --wgrad-stream $ws > $O/w1_ws${ws}_graph.log 2>&1 || exit $?
  grep '^{' $O/w1_ws${ws}_graph.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('w1 ws$ws', round(d['ms_per_step'],2))"
done
RANKS="0 1 2 3" TAG=5 bash scripts/gpu_r06_k.sh || exit $?
RANKS="3" TAG=5ws0 EXTRA="--wgrad-stream 0" bash scripts/gpu_r06_k.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_gc -o prof -- \
  python3 $R/benchmarks/bench_graphcast.py --mode step --steps 5 --warmup 2 --partition aligned \
  --rehearse-world 8 --rehearse-rank 3 --link-gbps 153 > $O/prof_w8r3.log 2>&1
echo "== prof rc=$?"
DB=$(find /tmp/prof_gc -name "*.db" | head -1)
python3 $R/scripts/prof_db_steps.py "$DB" --total-steps 8 --steps 4 --skip-last 1 --top 60 \
  > $O/prof_w8r3_aligned_kernels_per_step.txt
head -30 $O/prof_w8r3_aligned_kernels_per_step.txt | cut -c1-170
rm -rf /tmp/prof_gc
