#!/usr/bin/env bash
# Same-box A/B of source trees (each with its own in-tree _C.so): for every TREES entry
# (name:dir, "." = this tree) run the GEMM tests, the fp32 kernel timings and the 1-GPU
# headline step. Stops at the first fault-like exit. Outputs: gpurun_out/ab/<name>_*.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/ab
O=$R/gpurun_out/ab
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for spec in ${TREES:-cur:.}; do
  name=${spec%%:*}; d=${spec#*:}
  cd "$R/$d" || exit 1
  if [ "${TESTS:-1}" = 1 ]; then
    timeout -k 10 300 python -u -m pytest tests/test_f32_kernels_gpu.py -q -x --timeout 120 \
      --timeout-method thread -p no:cacheprovider -k "${TESTK:-gemm or dense_linear or fused_wide}" \
      > "$O/${name}_tests.log" 2>&1
    rc=$?; echo "== $name tests rc=$rc $(grep -E 'passed|failed' "$O/${name}_tests.log" | tail -1)"
    if fatal $rc || [ $rc != 0 ]; then exit $rc; fi
  fi
  if [ "${KERN:-1}" = 1 ]; then
    timeout -k 10 300 python -u benchmarks/bench_f32_kernels.py --reps 3 > "$O/${name}_kern.log" 2>&1
    rc=$?; echo "== $name kernels rc=$rc"; grep -E "^gemm|^wgrad" "$O/${name}_kern.log"
    if fatal $rc; then exit $rc; fi
  fi
  if [ "${HEAD:-1}" = 1 ]; then
    timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-extra ${EXTRA:-} \
      > "$O/${name}_bench.log" 2>&1
    rc=$?; echo "== $name bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$O/${name}_bench.log")"
    grep -o '"ms_max_over_ranks": {[^}]*}' "$O/${name}_bench.log"
    if fatal $rc; then exit $rc; fi
  fi
  cd "$R"
done
