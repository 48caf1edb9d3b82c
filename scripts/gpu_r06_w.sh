#!/bin/bash
# GraphCast event-joined branch measurements, then the full GPU suite + smoke + default bench.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash scripts/gpu_r06_v.sh || exit $?
bash scripts/gpu_r06_final.sh
