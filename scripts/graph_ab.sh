#!/usr/bin/env bash
# Eager vs whole-step HIP-graph replay (dgraph_amd.utils.graphed) on the launch-bound
# configurations: OGB GCN (arxiv shape), 3-layer SAGE (products shape at 1/10 and full),
# GraphCast (level-6 reference graph and a small level-4 one). Each GPU step has its own
# limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/graph_ab
mkdir -p "$OUT"
R=$OUT/results.jsonl
: > "$R"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -20 "$OUT/$name.log"; exit $rc; fi
  grep '^{' "$OUT/$name.log" | tail -1 | sed "s/^{/{\"run\": \"$name\", /" >> "$R"
}
timeout -k 10 300 python -u -m pytest tests/test_graphed_gpu.py -x -v --timeout 120 \
  --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
echo "pytest ok"
for g in "" "--cuda-graph"; do
  n=${g:+_graph}
  step products_s01$n 300 python -u bench.py --shape ogbn-products --scale 0.1 --steps 20 --warmup 3 --no-extra $g
  step products$n 300 python -u bench.py --shape ogbn-products --steps 10 --warmup 3 --no-extra $g
  step graphcast_l4$n 300 python -u benchmarks/bench_graphcast.py --mesh-level 4 --grid 181x360 --steps 20 --warmup 3 $g
  step graphcast$n 300 python -u benchmarks/bench_graphcast.py --steps 10 --warmup 3 $g
done
for g in "" "--cuda_graph"; do
  n=${g:+_graph}
  timeout -k 10 300 python -u -m dgraph_amd.experiments.ogb_gcn --dataset arxiv --epochs 30 \
    --log_dir "$OUT/gcn$n" $g > "$OUT/gcn$n.log" 2>&1 || { tail -20 "$OUT/gcn$n.log"; exit 1; }
  echo "gcn$n: $(cat "$OUT"/gcn$n/*runtime_experiment.log)"
done
cat "$R"
