#!/usr/bin/env bash
# link-delay tests (incl. streamed halos), structureless rehearsals (streamed), batch3
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4d
O=gpurun_out/r4d
timeout -k 10 300 python -u -m pytest tests/test_linkdelay_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "== pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest.log | tail -5
case $rc in 124|134|137|139) exit $rc;; esac
TESTS=0 RUNS="8:153 4:153" EXTRA="--global-frac 1.0" bash scripts/r4_ab.sh
bash scripts/r4_batch3.sh
