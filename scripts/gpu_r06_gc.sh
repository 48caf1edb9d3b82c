#!/bin/bash
# Round 6: GraphCast per-rank efficiency at W=8 — eager vs HIP-graph replay of the whole
# step, rehearsal ranks 0 and 7 behind the 153 GB/s link model, W=1 for reference; then a
# kernel trace of the W=8 rank-0 step (per-kernel totals).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/gc
O=gpurun_out/r06/gc
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <args...>
  local name=$1; shift
  timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --steps 20 --warmup 3 "$@" \
    > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep '^{' $O/$name.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(round(d['ms_per_step'],2), d.get('launch'), d.get('halo_rows'), d.get('regions_ms'))" || tail -5 $O/$name.log
  if fatal $rc; then exit $rc; fi
}
run w1_eager
run w1_graph --cuda-graph
run w8r0_g153_eager --rehearse-world 8 --rehearse-rank 0 --link-gbps 153
run w8r0_g153_graph --rehearse-world 8 --rehearse-rank 0 --link-gbps 153 --cuda-graph
run w8r7_g153_graph --rehearse-world 8 --rehearse-rank 7 --link-gbps 153 --cuda-graph
run w8r0_g0_graph --rehearse-world 8 --rehearse-rank 0 --cuda-graph
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_w8r0 -o prof -- \
    python3 $R/benchmarks/bench_graphcast.py --mode step --steps 5 --warmup 2 \
    --rehearse-world 8 --rehearse-rank 0 --link-gbps 153 > $R/$O/prof_w8r0.log 2>&1
  echo "== prof rc=$?"
fi
