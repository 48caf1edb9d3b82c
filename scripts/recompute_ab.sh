#!/usr/bin/env bash
# Halo recomputation: GPU numerics test, then per-rank compute and peak memory of the
# papers100M partition at W=2 and W=4 (loopback exchange), recompute off vs on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/recompute_ab
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_halo_recompute_gpu.py -x -v --timeout 200 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for w in ${WORLDS:-2 4}; do
  for mode in off on; do
    timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --rehearse-world $w \
      --rehearse-rank 1 --halo-recompute $mode > $OUT/reh_w${w}_$mode.log 2>&1 \
      || { tail -20 $OUT/reh_w${w}_$mode.log; exit 1; }
    grep '^{' $OUT/reh_w${w}_$mode.log
  done
done
