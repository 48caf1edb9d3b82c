#!/usr/bin/env bash
# W=1 headline step vs the fused executor's chunk rows (the chunk arena is the plan's only
# elastic buffer: peak memory vs step time). Output: gpurun_out/chunk_ab/*.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/chunk_ab
for cr in ${CRS:-0 1048576 524288 262144}; do
  DGRAPH_FUSED_CHUNK_ROWS=$cr timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-extra \
    > gpurun_out/chunk_ab/cr$cr.log 2>&1
  rc=$?
  python3 -c "
import json,sys
for l in open('gpurun_out/chunk_ab/cr$cr.log'):
    if l.startswith('{'):
        d=json.loads(l); print('cr=$cr', round(d['ms_per_step'],1), 'peak', d['peak_mem_gb_rank0'], d['config']['schedule']['chunk_rows'])"
  case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
done
