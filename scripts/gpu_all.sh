#!/usr/bin/env bash
# The whole GPU test suite WITHOUT -x (every failure listed), then smoke.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_all.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/pytest_gpu_all.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK
