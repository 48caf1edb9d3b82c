#!/bin/bash
# Full GPU test suite (no -x: every test runs and is reported) + smoke, on the GPU box.
# Usage: bash scripts/gpu_suite.sh [pytest selection...]
set -o pipefail
mkdir -p gpurun_out
sel=${@:-tests}
timeout -k 10 1000 python -u -m pytest $sel -m gpu -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gpu_suite.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_suite.log
grep -E "FAILED|ERROR" gpurun_out/gpu_suite.log | head -40
# a GPU fault / abort / timeout ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
tail -3 gpurun_out/smoke.log
echo "pytest rc=$rc smoke rc=$src"
exit $(( rc > src ? rc : src ))
