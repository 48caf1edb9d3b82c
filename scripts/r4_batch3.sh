#!/usr/bin/env bash
# Rehearsals W=2/4 (final kernels), products hidden-128 and papers100M hidden-512 (W=4 rank)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4c
O=gpurun_out/r4c
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -E '^\{' "$O/$name.log" | cut -c1-900
  if fatal $rc; then echo "FATAL at $name"; exit $rc; fi
}
TESTS=0 RUNS="${RUNS:-4:153 2:153}" bash scripts/r4_ab.sh
step products_h128 400 python -u bench.py --shape ogbn-products --hidden 128 --steps 5 --warmup 2 --no-extra
step products_h256 400 python -u bench.py --shape ogbn-products --hidden 256 --steps 5 --warmup 2 --no-extra
step papers_h512_w4 500 python -u bench.py --hidden 512 --rehearse-world 4 --link-gbps 153 --steps 3 --warmup 1 --no-extra
