#!/usr/bin/env bash
# A/B of the fused fp32 headline step: two-stream pipeline on/off, allocator config unset;
# then the fp32/bf16 ratio runs (products whole graph, papers100M W=4 rank 1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/ab1
summ() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', round(d['ms_per_step'],1), d['peak_mem_gb_rank0'], d.get('allocator_in_timed_steps'), json.dumps(d.get('regions',{}).get('ms_max_over_ranks')))"; }
DGRAPH_FUSED_PIPELINE=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extra > gpurun_out/ab1/pipe0.log 2>&1 || { tail -20 gpurun_out/ab1/pipe0.log; exit 1; }
summ gpurun_out/ab1/pipe0.log pipeline_off
PYTORCH_ALLOC_CONF= timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extra > gpurun_out/ab1/noconf.log 2>&1 || { tail -20 gpurun_out/ab1/noconf.log; exit 1; }
summ gpurun_out/ab1/noconf.log alloc_conf_unset
timeout -k 10 900 bash scripts/fp32_runs.sh
