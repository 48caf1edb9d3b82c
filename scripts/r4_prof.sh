#!/usr/bin/env bash
# Kernel traces: W=1 headline (2 timed steps) and one W-way rehearsal rank (link model).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4prof
O=$R/gpurun_out/r4prof
prof() {  # prof <tag> <bench args...>
  local tag=$1; shift
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$tag" -o run \
    -- python3 "$R/bench.py" "$@" > "$O/$tag.stdout.log" 2>&1
  local rc=$?
  cd "$R"
  echo "== $tag rc=$rc"
  python3 scripts/prof_summary.py "$O/$tag" 30 > "$O/$tag.summary.txt" 2>&1
  head -20 "$O/$tag.summary.txt"
  case $rc in 124|134|137|139) exit $rc;; esac
}
for spec in ${PROFS:-w1 w8}; do
  case $spec in
    w1) prof w1 --steps 2 --warmup 1 --no-extra ;;
    w*) prof $spec --rehearse-world ${spec#w} --link-gbps 153 --steps 2 --warmup 1 --no-extra ;;
  esac
done
