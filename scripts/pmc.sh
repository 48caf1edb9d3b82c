#!/usr/bin/env bash
# PMC counter pass (kernel-trace only, no sys/runtime trace domains).
# usage: COUNTERS="FETCH_SIZE TCC_HIT_sum" TAG=x bash scripts/pmc.sh python3 benchmarks/bench_spmm.py ...
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_${TAG:-run}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=("$@")
for i in "${!ARGS[@]}"; do
  case "${ARGS[$i]}" in benchmarks/*|bench.py|scripts/*) ARGS[$i]="$R/${ARGS[$i]}";; esac
done
timeout -k 10 ${TMO:-600} rocprofv3 --pmc ${COUNTERS:-FETCH_SIZE} --kernel-trace --output-format csv \
  -d "$OUT" -o run -- "${ARGS[@]}" > "$OUT/stdout.log" 2>&1
rc=$?
echo "pmc rc=$rc"
exit $rc
