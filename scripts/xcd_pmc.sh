#!/usr/bin/env bash
# L2 hit rate of the fp32 row-group SpMM with and without the XCD-contiguous block remap
# (one rocprofv3 --pmc pass per setting). Output: gpurun_out/xcd_pmc/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/xcd_pmc
O=gpurun_out/xcd_pmc
for PC in ${PCS:-16 32}; do for X in 0 1; do
  P="python3 $R/benchmarks/bench_f32_kernels.py --reps 1 --spmm-only --pass-cols $PC --xcd $X"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
     --kernel-trace --output-format csv -d "$R/$O/pc${PC}xcd$X" -o run -- $P > "$R/$O/pc${PC}xcd$X.log" 2>&1)
  rc=$?; echo "== pc$PC xcd$X rc=$rc"
  python3 scripts/pmc_summary.py $O/pc${PC}xcd$X "spmm_f32_rowgroup_kernel<int, " > $O/pc${PC}xcd$X.txt 2>&1
  head -4 $O/pc${PC}xcd$X.txt
  case $rc in 124|134|137|139) exit $rc;; esac
done; done
