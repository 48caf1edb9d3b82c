#!/bin/bash
# RGAT GPU tests (kernels, W=2 on one GPU with the layer-0 remake), the hidden-512
# streamed no-fill case at the tight gate, then the RGAT rank-1 W=8 rehearsal.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
O=gpurun_out/r06
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_rgat_lean.py "tests/test_multiproc_gpu.py::test_bench_step_hidden512_two_processes" \
  > $O/gpu_tests_d.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -4 $O/gpu_tests_d.log
case $rc in 0) ;; *) grep -E "^FAILED|Error" $O/gpu_tests_d.log | head; exit $rc;; esac
timeout -k 10 900 python -u benchmarks/bench_rgcn.py --model rgat --rehearse-world 8 \
  --rehearse-rank 1 --link-gbps 153 --steps 3 --warmup 1 > $O/rgat_w8r1_g153.out 2> $O/rgat_w8r1_g153.err
rc=$?; echo "== rgat w8r1 rc=$rc"; tail -2 $O/rgat_w8r1_g153.out; [ $rc -ne 0 ] && grep -i "error" $O/rgat_w8r1_g153.err | tail -3
exit 0
