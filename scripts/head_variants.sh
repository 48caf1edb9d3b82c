#!/usr/bin/env bash
# 1-GPU headline under knob variants on one box: VARS="name:ENV=V,ENV2=V2 ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/w1var
for spec in ${VARS:-base:}; do
  name=${spec%%:*}; envs=${spec#*:}
  ( export $(echo $envs | tr ',' ' ') ; timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-extra ${EXTRA:-} > gpurun_out/w1var/$name.log 2>&1 )
  rc=$?
  echo "== $name ($envs) rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/w1var/$name.log) $(grep -o '"chunk_rows": [0-9]*' gpurun_out/w1var/$name.log)"
  grep -o '"ms_max_over_ranks": {[^}]*}' gpurun_out/w1var/$name.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
