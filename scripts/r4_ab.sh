#!/usr/bin/env bash
# A/B of the W-way rehearsal: link delay on/off, interior-first on/off, plus a kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4ab
O=gpurun_out/r4ab
W=${W:-8}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <args...>
  local name=$1; shift
  timeout -k 10 400 python -u bench.py --rehearse-world $W --steps 3 --warmup 1 --no-extra "$@" \
      > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep '"rehearsal"' $O/$name.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['regions']['ms_max_over_ranks']
    print(round(d['ms_per_step_compute_loopback'],1), d.get('allocator_in_timed_steps'), {k:round(v,1) for k,v in r.items()})"
  if fatal $rc; then exit $rc; fi
}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_f32_kernels_gpu.py tests/test_linkdelay_gpu.py \
      tests/test_multiproc_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider \
      > $O/pytest.log 2>&1
  rc=$?; echo "== pytest rc=$rc"; tail -3 $O/pytest.log
  if fatal $rc; then exit $rc; fi
fi
run link153 --link-gbps 153
run link0
run link153_noif --link-gbps 153 --no-interior-first
run link0_noif --no-interior-first
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run \
    -- python3 "$R/bench.py" --rehearse-world $W --steps 2 --warmup 1 --no-extra --link-gbps 153 \
    > "$R/$O/prof_stdout.log" 2>&1
  echo "prof rc=$?"
  cd "$R"
  python3 scripts/prof_summary.py $O/prof 25 > $O/prof_summary.txt 2>&1; head -30 $O/prof_summary.txt
fi
