#!/usr/bin/env bash
# W-way rehearsals of the headline step, one rank on one GPU with the link-delayed loopback
# exchange (bench.py --rehearse-world W --link-gbps G): RUNS="W:GBPS[:HWQ] ..." (GBPS 0 = no
# delay; HWQ = DGRAPH_HW_QUEUES), EXTRA = more bench.py args (e.g. --global-frac 1.0),
# TESTS=1 runs the fp32 / link-delay / multi-process GPU tests first.
# Output: gpurun_out/rehearse/*.log, all.jsonl (one "rehearsal" JSON line per run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/rehearse
O=gpurun_out/rehearse
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <W> <args...>
  local name=$1 W=$2; shift 2
  timeout -k 10 500 python -u bench.py --rehearse-world $W --steps 3 --warmup 1 --no-extra "$@" \
      > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep '"rehearsal"' $O/$name.log >> $O/all.jsonl
  grep '"rehearsal"' $O/$name.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['regions']['ms_max_over_ranks']
    print(round(d['ms_per_step_compute_loopback'],1), d.get('peak_mem_gb'), d.get('allocator_in_timed_steps'), d.get('schedule'), {k:round(v,1) for k,v in r.items()})"
  if fatal $rc; then exit $rc; fi
}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest ${TESTFILES:-tests/test_f32_kernels_gpu.py tests/test_linkdelay_gpu.py tests/test_multiproc_gpu.py} \
      -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
  rc=$?; echo "== pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest.log | tail -8
  if fatal $rc; then exit $rc; fi
fi
for spec in ${RUNS:-8:153 8:0 2:153 4:153}; do
  # W:GBPS[:HWQ]
  W=${spec%%:*}; rest=${spec#*:}; G=${rest%%:*}; Q=${rest#*:}
  [ "$Q" = "$rest" ] && Q=""
  if [ -n "$Q" ]; then
    DGRAPH_HW_QUEUES=$Q run w${W}_g${G}_q${Q} $W --link-gbps $G ${EXTRA:-}
  else
    run w${W}_g${G} $W --link-gbps $G ${EXTRA:-}
  fi
done
