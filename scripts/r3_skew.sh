#!/usr/bin/env bash
# Rank-skew rehearsals of the headline step (fp32 fused executor): one rank's compute with a
# loopback exchange per run. PAIRS="W:r W:r ..." (default: W=2 and W=4 ranks 0 and W-1).
# Appends one JSON line per run to gpurun_out/rehearse_allranks.jsonl.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/skew
PAIRS=${PAIRS:-"2:0 2:1 4:0 4:3"}
for pr in $PAIRS; do
  w=${pr%%:*}; r=${pr##*:}
  log=gpurun_out/skew/reh_w${w}_r${r}_gf${GF:-0.05}.log
  timeout -k 10 ${TMO:-420} python -u bench.py --steps 3 --warmup 1 --no-extra \
    --global-frac ${GF:-0.05} --rehearse-world $w --rehearse-rank $r > $log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "w=$w r=$r rc=$rc"; tail -20 $log; exit $rc; fi
  grep '^{' $log | tee -a gpurun_out/rehearse_allranks.jsonl | cut -c1-220
done
