#!/usr/bin/env bash
# SpMM kernel A/B on the papers100M shape (+ the GPU SpMM tests first).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "spmm or sage" --timeout 120 --timeout-method thread > gpurun_out/spmm_tests.log 2>&1
for m in ${MEANS:-row}; do for w in ${WINDOWS:-16384}; do
  timeout -k 10 300 python benchmarks/bench_spmm.py --shape ogbn-papers100M --feats ${FEATS:-128,256} \
    --rounds ${ROUNDS:-3} --variants ${VARIANTS:-2:2:128,3:2:128} --window $w --mean $m > gpurun_out/spmm_ab_${m}_w$w.log 2>&1
done; done
