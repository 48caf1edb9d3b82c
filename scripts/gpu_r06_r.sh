#!/bin/bash
# Structureless W=2 rank at 153 GB/s: the planner's memory decisions, default vs the
# S-compacted transposed adjacency forced on.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/w2ts
O=gpurun_out/r06/w2ts
for ts in auto on; do
  DGRAPH_FUSED_COMPACT_T=$ts timeout -k 10 600 python -u bench.py --rehearse-world 2 --global-frac 1.0 \
    --link-gbps 153 --steps 3 --warmup 1 --no-extra > $O/w2_ts_$ts.log 2>&1
  rc=$?; echo "== ts=$ts rc=$rc"
  grep '"rehearsal"' $O/w2_ts_$ts.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); s=d['schedule']
    print(round(d['ms_per_step_compute_loopback'],1), d.get('peak_mem_gb'), {k:round(v,1) for k,v in d['regions']['ms_max_over_ranks'].items()})
    for m in s.get('memory_plan', []): print('   ', m)"
  case $rc in 0) ;; *) tail -5 $O/w2_ts_$ts.log; exit $rc;; esac
done
