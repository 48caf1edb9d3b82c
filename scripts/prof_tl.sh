#!/usr/bin/env bash
# Kernel-trace timeline of one W-way rehearsal rank (link model on): gpurun_out/tl_*/
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
W=${W:-8}
OUT=$R/gpurun_out/tl_w$W
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${TMO:-500} rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run \
  -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-extra --rehearse-world $W \
  --link-gbps ${GBPS:-153} ${EXTRA:-} > "$OUT/stdout.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
ms=$(grep -o '"ms_per_step_compute_loopback": [0-9.]*' "$OUT/stdout.log" | grep -o '[0-9.]*$')
echo "step ms=$ms"
python3 "$R/scripts/prof_timeline.py" "$OUT" "${ms:-1000}" ${ROWS:-400} > "$R/gpurun_out/tl_w$W.txt"
head -12 "$R/gpurun_out/tl_w$W.txt"
exit $rc
