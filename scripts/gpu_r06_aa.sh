#!/bin/bash
# Final tree: bench.py through torchrun at W=2 and W=4 with every rank on the one GPU (RCCL
# socket transport), with the one-sided probe child job (mode: host on a shared GPU).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
for W in 2 4; do
  DGRAPH_RCCL_SHARED_GPU=1 timeout -k 10 500 python -u bench.py --gpus $W --scale 0.02 --steps 2 \
    --warmup 1 --no-extra > gpurun_out/r06/bench_w${W}_shared_final.json 2> gpurun_out/r06/bench_w${W}_shared_final.err
  rc=$?; echo "== W=$W rc=$rc"
  case $rc in 0) ;; *) tail -20 gpurun_out/r06/bench_w${W}_shared_final.err; exit $rc;; esac
  python3 -c "
import json;d=json.loads(open('gpurun_out/r06/bench_w${W}_shared_final.json').read().splitlines()[-1])
p=d.get('shmem_probe',{}); print(d['ms_per_step'], d['n_gpus'], json.dumps({k:p.get(k) for k in ('mode','child_wall_s','failed')}), json.dumps({k:(p.get(k) or {}).get('bitwise_equal_to_torch') for k in ('put_rows','remote_gather')}))"
done
