#!/bin/bash
# Full GPU suite + smoke, then the default bench.py (N=1) on this tree.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash scripts/gpu_suite.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
brc=$?
echo "== bench rc=$brc"; tail -c 600 gpurun_out/bench_default.json
exit $(( rc > brc ? rc : brc ))
