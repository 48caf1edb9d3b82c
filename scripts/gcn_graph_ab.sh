set -o pipefail
OUT=gpurun_out/graph_ab
mkdir -p $OUT
for g in "" "--cuda_graph"; do
  n=${g:+_graph}
  timeout -k 10 300 python -u -m dgraph_amd.experiments.ogb_gcn --dataset arxiv --epochs 30 \
    --log_dir "$OUT/gcn$n" $g > "$OUT/gcn$n.log" 2>&1 || { tail -20 "$OUT/gcn$n.log"; exit 1; }
  echo "gcn$n: $(cat "$OUT"/gcn$n/*runtime_experiment.log) $(tail -1 $OUT/gcn$n/*test_results.log)"
done
GF=1.0 WORLDS="2 4" TMO=400 bash scripts/rehearse.sh
