#!/bin/bash
# RGAT per-head kernel passes: GPU tests, then the 1/8-scale step (plain and kernel-traced,
# summarised on the box) and the rank-1 W=8 rehearsal at 153 GB/s.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06
O=$R/gpurun_out/r06
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_rgat_lean.py > $O/gpu_tests_g.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -3 $O/gpu_tests_g.log
case $rc in 0) ;; *) grep -E "^FAILED|Error" $O/gpu_tests_g.log | head; exit $rc;; esac
timeout -k 10 900 python -u benchmarks/bench_rgcn.py --model rgat --scale 0.125 --steps 3 --warmup 1 \
  > $O/rgat_eighth_g.out 2> $O/rgat_eighth_g.err
rc=$?; echo "== eighth rc=$rc"; tail -1 $O/rgat_eighth_g.out | cut -c1-250
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u benchmarks/bench_rgcn.py --model rgat --rehearse-world 8 \
  --rehearse-rank 1 --link-gbps 153 --steps 3 --warmup 1 > $O/rgat_w8r1_g153_g.out 2> $O/rgat_w8r1_g153_g.err
rc=$?; echo "== w8r1 rc=$rc"; tail -1 $O/rgat_w8r1_g153_g.out | cut -c1-250
case $rc in 124|134|137|139) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace -d /tmp/prof_rgat -o prof -- \
  python3 $R/benchmarks/bench_rgcn.py --model rgat --scale 0.125 --steps 3 --warmup 1 \
  > $O/rgat_eighth_prof_g.out 2> $O/rgat_eighth_prof_g.err
echo "== prof rc=$?"
DB=$(find /tmp/prof_rgat -name "*.db" | head -1)
python3 $R/scripts/prof_db_steps.py "$DB" --total-steps 4 --steps 3 --top 40 > $O/rgat_eighth_kernels_per_step_g.txt
head -12 $O/rgat_eighth_kernels_per_step_g.txt | cut -c1-150
rm -rf /tmp/prof_rgat
