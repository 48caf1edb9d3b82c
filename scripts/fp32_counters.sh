#!/usr/bin/env bash
# PMC counter passes over the fp32 hot kernels at their step shapes
# (benchmarks/bench_f32_kernels.py: row-group SpMM, column-mapped SpMM, MFMA GEMM, weight
# gradient), one rocprofv3 --pmc run per counter group (each within the per-block counter
# limits), summarised per kernel by scripts/pmc_summary.py. Output: gpurun_out/pmc/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/pmc
O=gpurun_out/pmc
timeout -k 10 300 python -u benchmarks/bench_f32_kernels.py > $O/timings.log 2>&1
rc=$?; echo "== timings rc=$rc"; grep -E "^spmm|^gemm|^wgrad" $O/timings.log
case $rc in 124|134|137|139) exit $rc;; esac
P="python3 $R/benchmarks/bench_f32_kernels.py --reps 1"
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
         "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  mkdir -p $O/pass$i
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace \
     --output-format csv -d "$R/$O/pass$i" -o run -- $P > "$R/$O/pass$i.log" 2>&1)
  rc=$?; echo "== pass$i rc=$rc"
  python3 scripts/pmc_summary.py $O/pass$i spmm_f32 gemm_f32 wgrad_f32 > $O/pass$i.txt 2>&1
  head -12 $O/pass$i.txt
  case $rc in 124|134|137|139) exit $rc;; esac
done
