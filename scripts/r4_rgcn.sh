#!/usr/bin/env bash
# fp32 R-GCN (lean path): GPU tests, 1/8-scale step, W=8 rank-1 rehearsal, kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/rgcn
O=gpurun_out/rgcn
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -E '^\{|passed|failed|Error' "$O/$name.log" | cut -c1-900
  if fatal $rc; then echo "FATAL at $name"; exit $rc; fi
}
step tests 400 python -u -m pytest tests/test_rgcn.py tests/test_f32_kernels_gpu.py tests/test_graphcast.py tests/test_act_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "rgcn or dense_linear or graphcast or gemm or wgrad or act"
step eighth 500 python -u benchmarks/bench_rgcn.py --scale 0.125 --steps 3 --warmup 1
step gc73_mfma 300 python -u benchmarks/bench_graphcast.py --steps 10 --warmup 3
step gc73_lib 300 env DGRAPH_F32_LINEAR=0 python -u benchmarks/bench_graphcast.py --steps 10 --warmup 3
step eighth_lib 500 env DGRAPH_F32_LINEAR=0 python -u benchmarks/bench_rgcn.py --scale 0.125 --steps 3 --warmup 1
step w8r1 600 python -u benchmarks/bench_rgcn.py --rehearse-world 8 --rehearse-rank 1 --steps 3 --warmup 1 --backend rocshmem
step w8r1_exp 600 env PYTORCH_ALLOC_CONF=expandable_segments:True python -u benchmarks/bench_rgcn.py --rehearse-world 8 --rehearse-rank 1 --steps 3 --warmup 1 --backend rocshmem
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run \
    -- python3 "$R/benchmarks/bench_rgcn.py" --scale 0.125 --steps 2 --warmup 1 > "$R/$O/prof.log" 2>&1
  rc=$?; cd "$R"; echo "== prof rc=$rc"
  python3 scripts/prof_summary.py "$O/prof" 40 > "$O/prof_summary.txt" 2>&1; head -45 "$O/prof_summary.txt"
  find "$O/prof" -name "*kernel_stats.csv" -exec cp {} "$O/" \;
  rm -rf "$O/prof"
fi
