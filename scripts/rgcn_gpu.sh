#!/usr/bin/env bash
# R-GCN (BASELINE config 4) on one MI355X. Steps (RUNS, space-separated; default all but prof):
#   tests     GPU tests of the R-GCN / fp32 linear paths
#   eighth    1/8-scale MAG240M (the per-GPU share of the 8-GPU job), for each PATHS entry
#   w8r1      rank 1 of the real 8-way partition (loopback exchange)
#   prof      rocprofv3 kernel stats of the 1/8-scale step, for each PATHS entry
# PATHS: lean / aggregate-first / auto (bench_rgcn.py --path); DTYPE fp32|bf16; env passes
# through (e.g. DGRAPH_F32_LINEAR=0 for library GEMMs). Outputs: gpurun_out/rgcn/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/rgcn
O=gpurun_out/rgcn
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -E '^\{|passed|failed|Error' "$O/$name.log" | cut -c1-900
  if fatal $rc; then echo "FATAL at $name"; exit $rc; fi
}
S=benchmarks/bench_rgcn.py
B="$S --dtype ${DTYPE:-fp32}"
for run in ${RUNS:-tests eighth w8r1}; do
  case $run in
    tests) step tests 400 python -u -m pytest tests/test_rgcn.py tests/test_f32_kernels_gpu.py \
             tests/test_act_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
             -p no:cacheprovider -k "rgcn or dense_linear or act" ;;
    eighth) for p in ${PATHS:-auto}; do
              step eighth_$p 500 python -u $B --path $p --scale 0.125 --steps 3 --warmup 1; done ;;
    w8r1) step w8r1 600 python -u $B --rehearse-world 8 --rehearse-rank 1 --steps 3 --warmup 1 \
            --backend ${BACKEND:-rocshmem} ;;
    prof) for p in ${PATHS:-auto}; do
            cd /tmp && export TMPDIR=/tmp
            timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
              -d "$R/$O/prof_$p" -o run -- python3 "$R/$S" --dtype ${DTYPE:-fp32} --path $p --scale 0.125 --steps 2 \
              --warmup 1 > "$R/$O/prof_$p.log" 2>&1
            rc=$?; cd "$R"; echo "== prof_$p rc=$rc"
            python3 scripts/prof_summary.py "$O/prof_$p" 40 > "$O/prof_$p.txt" 2>&1
            head -30 "$O/prof_$p.txt"
            find "$O/prof_$p" -name "*kernel_stats.csv" -exec cp {} "$O/prof_${p}_kernel_stats.csv" \;
            rm -rf "$O/prof_$p"
            if fatal $rc; then exit $rc; fi
          done ;;
  esac
done
