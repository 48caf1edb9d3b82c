#!/usr/bin/env bash
# Kernel-trace timeline of the last WIN ms of an arbitrary python command:
#   TAG=name WIN=ms CMD="benchmarks/x.py args" bash scripts/prof_tl_cmd.sh
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/tl_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${TMO:-500} rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run \
  -- python3 $R/$CMD > "$OUT/stdout.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
python3 "$R/scripts/prof_timeline.py" "$OUT" "$WIN" ${ROWS:-400} > "$R/gpurun_out/tl_$TAG.txt"
head -14 "$R/gpurun_out/tl_$TAG.txt"
exit $rc
