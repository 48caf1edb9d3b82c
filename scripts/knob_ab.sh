#!/usr/bin/env bash
# A/B of one executor knob (KNOB, default DGRAPH_FUSED_PACK_STREAM) over VALS (default
# "comm compute") in W-way link-model rehearsals: SPECS="W:global_frac ...".
# Output: gpurun_out/pack_ab/*.log, all.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/${OUTD:-pack_ab}
O=gpurun_out/${OUTD:-pack_ab}
KNOB=${KNOB:-DGRAPH_FUSED_PACK_STREAM}
for spec in ${SPECS:-8:0.05 2:0.05 8:1.0}; do
  W=${spec%%:*}; gf=${spec#*:}
  for ps in ${VALS:-comm compute}; do
    name=w${W}_gf${gf}_$ps
    env $KNOB=$ps timeout -k 10 ${TMO:-500} python -u bench.py --rehearse-world $W \
        --steps 3 --warmup 1 --no-extra --link-gbps 153 --global-frac $gf > $O/$name.log 2>&1
    rc=$?
    echo "== $name rc=$rc"
    grep '"rehearsal"' $O/$name.log | sed "s/^{/{\"knob\": \"$KNOB=$ps\", /" >> $O/all.jsonl
    grep '"rehearsal"' $O/$name.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['regions']
    print(round(d['ms_per_step_compute_loopback'],1), 'exposed', r.get('exposed_exchange_ms_max'), {k:round(v,1) for k,v in r['ms_max_over_ranks'].items()})"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
