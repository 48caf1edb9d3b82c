#!/usr/bin/env bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters in this pass).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_${TAG:-run}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${TMO:-900} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
  -- python3 "$R/${SCRIPT:-bench.py}" ${BENCH_ARGS:---steps 2 --warmup 1} > "$OUT/stdout.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
find "$OUT" -name "*kernel_stats.csv" | head -3
f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -25 "$f" | cut -c1-220
exit $rc
