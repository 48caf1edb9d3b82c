#!/usr/bin/env python3
"""Offline halo-plan generation for a W-rank OGB run (experiments/OGB/GenerateCache.py).

Builds every rank's CommunicationPattern in one process (no process group, no GPUs) and
saves ``{out}/{dataset}_rank_{r}_of_{W}_comm_pattern.pt`` files (plain tensors, loadable
with ``torch.load(weights_only=True)``); ``examples/ogb/main.py`` ranks can load theirs
with :func:`dgraph_amd.plan.pattern.load_pattern` instead of building it collectively.

    python examples/ogb/generate_cache.py --dataset arxiv --world-size 8 --out plans
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="arxiv")
    ap.add_argument("--world-size", type=int, default=2)
    ap.add_argument("--out", default="plans")
    ap.add_argument("--root-dir", default="data")
    ap.add_argument("--scale", type=float, default=1.0, help="synthetic-graph scale")
    ap.add_argument("--node-rank-placement-file", default=None)
    ap.add_argument("--partitioner", default="round_robin",
                    help="round_robin | contiguous | random | label_propagation | metis")
    a = ap.parse_args(argv)
    from dgraph_amd.data.ogbn import _load_ogb, _synthetic_ogb
    from dgraph_amd.data.partition import partition, partition_stats
    from dgraph_amd.plan.pattern import build_all_patterns_offline, save_patterns

    name = a.dataset if a.dataset.startswith("ogbn-") else f"ogbn-{a.dataset}"
    try:
        graph, _, _ = _load_ogb(name, a.root_dir)
    except Exception:  # noqa: BLE001 - no ogb / no network: synthetic graph of that shape
        graph, _, _ = _synthetic_ogb(name, scale=a.scale)
    edge_index = torch.as_tensor(graph["edge_index"]).long()
    V = int(graph["num_nodes"])
    if a.node_rank_placement_file:
        part = torch.load(a.node_rank_placement_file, weights_only=True).long()
    else:
        part = partition(a.partitioner, V, a.world_size, edge_index=edge_index)
    # (central, neighbour) pairs of the symmetrised graph, duplicates removed
    E = torch.unique(torch.cat([edge_index.t(), edge_index.flip(0).t()], 0), dim=0)
    pats = build_all_patterns_offline(E, part, a.world_size)
    paths = save_patterns(pats, a.out, name)
    print(partition_stats(edge_index, part, a.world_size))
    for cp, p in zip(pats, paths):
        print(p, cp.stats())
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
