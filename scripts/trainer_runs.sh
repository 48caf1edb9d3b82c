#!/usr/bin/env bash
# End-to-end training runs of the three reference applications on one MI355X (synthetic
# data of the reference shapes): OGB GCN (arxiv shape, 30 epochs), OGB-LSC RGAT and R-GCN
# (synthetic MAG-like graph), GraphCast (20 iterations). Per-epoch JSONL metrics and the
# reference log files land under gpurun_out/train_*.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m dgraph_amd.experiments.ogb_gcn --dataset arxiv --epochs 30 \
  --log_dir $O/train_gcn --metrics_jsonl $O/train_gcn/metrics.jsonl > $O/train_gcn.log 2>&1
tail -3 $O/train_gcn.log
for m in rgat rgcn; do
  timeout -k 10 300 python -u -m dgraph_amd.experiments.ogb_lsc --model $m --num_papers 65536 \
    --num_authors 131072 --num_institutions 512 --num_features 128 --hidden_channels 128 \
    --heads 4 --epochs 40 --lr 1e-3 --log_dir $O/train_$m \
    --metrics_jsonl $O/train_$m/metrics.jsonl > $O/train_$m.log 2>&1
  tail -3 $O/train_$m.log
done
timeout -k 10 400 python -u -m dgraph_amd.experiments.graphcast --iters 20 --dtype bf16 \
  --log_dir $O/train_graphcast --metrics_jsonl $O/train_graphcast/metrics.jsonl \
  > $O/train_graphcast.log 2>&1
tail -3 $O/train_graphcast.log
