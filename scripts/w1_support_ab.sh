#!/usr/bin/env bash
# One GPU, papers100M full-graph step: persistent ReLU-mask buffers, with and without the
# gradient support of the layer below the output layer (DGRAPH_BENCH_GRAD_SUPPORT).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/w1_support
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_precision_gpu.py tests/test_determinism.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for gs in auto on; do
  DGRAPH_BENCH_GRAD_SUPPORT=$gs timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-extra > $OUT/bench_$gs.log 2>&1 || { tail -20 $OUT/bench_$gs.log; exit 1; }
  echo "support=$gs $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$gs.log | head -1) $(grep -o '"edges_aggregated_per_step": [0-9.e+]*' $OUT/bench_$gs.log | head -1) $(grep -o '"final_loss": [0-9.]*' $OUT/bench_$gs.log) $(grep -o '"peak_mem_gb_rank0": [0-9.]*' $OUT/bench_$gs.log)"
done
