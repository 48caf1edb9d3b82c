#!/usr/bin/env bash
# Gradient support of the layer below the output layer (prepared on partitioned graphs):
# GPU numerics tests, the 1-GPU headline step (support not prepared there), and one rank
# of the W=2 / W=4 / W=8 partitions with support on vs off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/support_ab
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_precision_gpu.py tests/test_halo_recompute_gpu.py tests/test_row_scale_colsum_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-extra > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
echo "1 GPU: $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench.log | head -1) $(grep -o '"peak_mem_gb_rank0": [0-9.]*' $OUT/bench.log)"
for w in ${WORLDS:-2 4 8}; do
  for v in 1 0; do
    DGRAPH_GRAD_SUPPORT=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --rehearse-world $w --rehearse-rank 1 > $OUT/reh${w}_$v.log 2>&1 || { tail -20 $OUT/reh${w}_$v.log; exit 1; }
    echo "W=$w support=$v $(grep -o '"ms_per_step_compute_loopback": [0-9.]*' $OUT/reh${w}_$v.log) $(grep -o '"peak_mem_gb": [0-9.]*' $OUT/reh${w}_$v.log) $(grep -o '"final_loss_local": [0-9.]*' $OUT/reh${w}_$v.log)"
  done
done
