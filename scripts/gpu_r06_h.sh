#!/bin/bash
# RGAT with whole-row attention passes and batched narrow GEMMs (1/8 scale, rank-1 W=8 at
# 153 GB/s), then the default W=1 headline bench on this tree.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
O=$R/gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_rgat_lean.py tests/test_act_gpu.py > $O/gpu_tests_h.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -2 $O/gpu_tests_h.log
case $rc in 0) ;; *) grep -E "^FAILED|Error" $O/gpu_tests_h.log | head; exit $rc;; esac
timeout -k 10 900 python -u benchmarks/bench_rgcn.py --model rgat --scale 0.125 --steps 3 --warmup 1 \
  > $O/rgat_eighth_h.out 2> $O/rgat_eighth_h.err
rc=$?; echo "== eighth rc=$rc"; tail -1 $O/rgat_eighth_h.out | cut -c1-250
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u benchmarks/bench_rgcn.py --model rgat --rehearse-world 8 \
  --rehearse-rank 1 --link-gbps 153 --steps 3 --warmup 1 > $O/rgat_w8r1_g153_h.out 2> $O/rgat_w8r1_g153_h.err
rc=$?; echo "== w8r1 rc=$rc"; tail -1 $O/rgat_w8r1_g153_h.out | cut -c1-250
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u bench.py > $O/bench_default_h.json 2> $O/bench_default_h.err
rc=$?; echo "== bench rc=$rc"; python3 -c "
import json;d=json.loads(open('$O/bench_default_h.json').read().splitlines()[-1])
print(d['ms_per_step'], d['value'], d['peak_mem_gb_rank0'], d.get('structureless',{}).get('ms_per_step'), d.get('bf16_stack',{}).get('ms_per_step'))"
timeout -k 10 400 env DGRAPH_RCCL_SHARED_GPU=1 python -u bench.py --gpus 2 --scale 0.02 --steps 2 \
  --warmup 1 --no-extra > $O/bench_w2_shared_h.json 2> $O/bench_w2_shared_h.err
rc=$?; echo "== w2 shared rc=$rc"
python3 -c "import json;d=json.loads(open('$O/bench_w2_shared_h.json').read().splitlines()[-1]);print(json.dumps(d['shmem_probe']))" | cut -c1-1500
