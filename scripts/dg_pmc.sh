#!/usr/bin/env bash
# dual-GEMM timing (both kernels) + counter passes on the B-stationary kernel
set -eu
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
SH=${SHAPES:-256:128:128,256:256:256,192:256:0,256:192:0}
timeout -k 10 400 python -u benchmarks/bench_dual_gemm.py --rows ${ROWS:-111059956} --variants 1,2 --no-library --shapes $SH > gpurun_out/dg_ab.log 2>&1
grep -v '^{' gpurun_out/dg_ab.log
[ -n "${NOPMC:-}" ] && exit 0
P="python3 benchmarks/bench_dual_gemm.py --rows 33554432 --variants 2 --no-library --shapes $SH"
COUNTERS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" TAG=dg_sq TMO=120 bash scripts/pmc.sh $P
COUNTERS="FETCH_SIZE" TAG=dg_fetch TMO=120 bash scripts/pmc.sh $P
COUNTERS="WRITE_SIZE GRBM_GUI_ACTIVE" TAG=dg_write TMO=120 bash scripts/pmc.sh $P
for t in dg_sq dg_fetch dg_write; do python3 scripts/pmc_summary.py gpurun_out/pmc_$t dual_gemm_bs > gpurun_out/pmc_$t.txt; done
cat gpurun_out/pmc_dg_sq.txt | head -60
