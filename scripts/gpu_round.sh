#!/usr/bin/env bash
# GPU session: GPU tests, the 1-GPU headline, link-delayed rehearsals of W = 2/4/8.
# Stops at the first fault-like exit (timeout / abort / segfault); plain test failures go on.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/round
O=gpurun_out/round
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.log"
  if fatal $rc; then echo "FATAL at $name"; exit $rc; fi
  return 0
}
TESTS=${TESTS:-tests}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 900 python -u -m pytest $TESTS -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
  grep -E "^FAILED|^ERROR|passed|failed" $O/pytest_gpu.log | tail -20
fi
if [ "${SKIP_W1:-0}" != 1 ]; then
  step bench_w1 600 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-extra
fi
for W in ${WORLDS:-2 4 8}; do
  step rehearse_w$W 600 python -u bench.py --rehearse-world $W --rehearse-rank ${RRANK:-0} \
      --link-gbps ${GBPS:-153} --steps ${STEPS:-3} --warmup 1 --no-extra
  grep '"rehearsal"' $O/rehearse_w$W.log >> $O/rehearse_linkdelay.jsonl
done
echo DONE
