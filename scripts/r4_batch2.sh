#!/usr/bin/env bash
# fp32 kernel timings + PMC counter passes, fp32 R-GCN / GraphCast (configs 4/5), rehearsals.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4b
O=gpurun_out/r4b
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -E '^\{|^\[bench|rc=' "$O/$name.log" | tail -2 | cut -c1-600
  if fatal $rc; then echo "FATAL at $name"; exit $rc; fi
}
if [ "${KERN:-1}" = 1 ]; then
  step f32_kernels 300 python -u benchmarks/bench_f32_kernels.py
  P="python3 $R/benchmarks/bench_f32_kernels.py --reps 1"
  i=0
  for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    mkdir -p $O/pmc$i
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace \
       --output-format csv -d "$R/$O/pmc$i" -o run -- $P > "$R/$O/pmc$i.log" 2>&1)
    rc=$?; echo "== pmc$i rc=$rc"
    python3 scripts/pmc_summary.py $O/pmc$i spmm_f32 gemm_f32 wgrad_f32 > $O/pmc$i.txt 2>&1
    if fatal $rc; then exit $rc; fi
  done
fi
if [ "${MODELS:-1}" = 1 ]; then
  step rgcn_fp32_eighth 400 python -u benchmarks/bench_rgcn.py --scale 0.125 --steps 5 --warmup 2
  step rgcn_fp32_w8r1 400 python -u benchmarks/bench_rgcn.py --rehearse-world 8 --rehearse-rank 1 --steps 3 --warmup 1
  step gc_fp32_73 400 python -u benchmarks/bench_graphcast.py --mode step --dtype fp32
  step gc_fp32_227 400 python -u benchmarks/bench_graphcast.py --mode step --dtype fp32 --channel-config era5-37
fi
if [ "${REH:-1}" = 1 ]; then
  TESTS=0 RUNS="${RUNS:-8:153 4:153}" bash scripts/r4_ab.sh
fi
