#!/usr/bin/env bash
# A/B of the two-stream chunk pipeline (the co-residency probe shows it does not overlap),
# then rank-skew rehearsals of the fused fp32 step (one rank of a W-way partition each).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
DGRAPH_FUSED_PIPELINE=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extra > gpurun_out/nopipe.log 2>&1
rc=$?; grep '^{' gpurun_out/nopipe.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nopipe', d['ms_per_step'], json.dumps(d.get('regions',{}).get('ms_max_over_ranks')))"; [ $rc -eq 0 ] || exit $rc
PAIRS="8:0 8:3 8:7 2:0 2:1 4:0 4:3" TMO=300 bash scripts/r3_skew.sh
