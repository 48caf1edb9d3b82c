#!/usr/bin/env bash
# Same-box A/B of the 1-GPU headline: round-3 tree (abtree/r03) vs this tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/w1ab
for t in new old new; do
  if [ $t = old ]; then d=abtree/r03; else d=.; fi
  (cd $d && timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-extra ${EXTRA:-} > $R/gpurun_out/w1ab/$t.log 2>&1)
  rc=$?
  echo "== $t rc=$rc"
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/w1ab/$t.log
  grep -o '"regions": {"ms_max_over_ranks": {[^}]*}' gpurun_out/w1ab/$t.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
