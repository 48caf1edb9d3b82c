#!/usr/bin/env bash
# GPU-box check: smoke, GPU tests, short benches. Each GPU step has its own time limit;
# the script stops at the first fault/abort/timeout (exit >= 2 or signal codes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1

run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/summary.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/summary.log"
  tail -n 5 "$OUT/$name.log" | tee -a "$OUT/summary.log"
  if [ $rc -ge 2 ]; then echo "stopping after $name (rc=$rc)" | tee -a "$OUT/summary.log"; exit $rc; fi
  return 0
}

STEPS=${STEPS:-smoke,tests,bench_small,bench}
[[ $STEPS == *smoke* ]] && run smoke 400 python __graft_entry__.py smoke
[[ $STEPS == *tests* ]] && run pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
[[ $STEPS == *bench_small* ]] && run bench_products 600 python bench.py --shape ogbn-products --steps 5 --warmup 2 --verbose
[[ $STEPS == *bench,* || $STEPS == *bench ]] && run bench_papers 1000 python bench.py --steps 5 --warmup 2 --verbose
echo done
