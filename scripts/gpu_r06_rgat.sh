#!/bin/bash
# Round 6: RGAT lean path on the GPU (fused attention kernels vs fp64 CPU, bitwise), the
# one-sided heap kernels' device rates, and RGAT at MAG240M shape: one GPU's 1/8 share and
# rank 1 of the 8-way partition behind the 153 GB/s link model.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
O=gpurun_out/r06
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step <name> <timeout> <cmd...>: stdout -> $O/<name>.out, stderr -> $O/<name>.err
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"; tail -3 $O/$name.out
  if [ $rc -ne 0 ]; then tail -5 $O/$name.err; fi
  if fatal $rc; then exit $rc; fi
  return 0
}
step rgat_gpu_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  -m gpu tests/test_rgat_lean.py
grep -q " passed" $O/rgat_gpu_tests.out && ! grep -q "FAILED\|failed" $O/rgat_gpu_tests.out || exit 1
step bench_heap 300 python -u benchmarks/bench_heap.py
for sc in ${SCALES:-0.0625 0.125}; do
  step rgat_scale$sc 900 python -u benchmarks/bench_rgcn.py --model rgat --scale $sc --steps 3 --warmup 1
done
if [ "${REHEARSE:-1}" = 1 ]; then
  step rgat_w8r1_g153 900 python -u benchmarks/bench_rgcn.py --model rgat --rehearse-world 8 \
    --rehearse-rank 1 --link-gbps 153 --steps 3 --warmup 1
fi
