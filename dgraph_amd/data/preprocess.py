"""Renumbering and homogeneous-graph preprocessing (DGraph/data/preprocess.py).

* :func:`node_renumbering` — stable sort of vertices by owner rank so rank ``r`` owns a
  contiguous id range (invariant I1). Returns ``(new_to_old, sorted_rank_of_new)`` like
  the reference, plus :func:`inverse_permutation` for relabelling.
* :func:`edge_renumbering` — relabels edges into the new numbering and sorts them
  (stably) by the rank of their source vertex (I2).

Correction vs the reference: the reference relabelled edge endpoints and split indices
with the *new->old* permutation (``renumbered_nodes[src]``, preprocess.py:20-21,95-97)
where the *old->new* inverse is required; the two coincide only for involutive
permutations. Here relabelling always uses the inverse permutation.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from .graph import DistributedGraph


def inverse_permutation(perm: torch.Tensor) -> torch.Tensor:
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel(), device=perm.device, dtype=perm.dtype)
    return inv


def node_renumbering(node_rank_placement: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """-> (``new_to_old`` vertex permutation, owner rank of each new id, ascending)."""
    ranks_sorted, new_to_old = torch.sort(node_rank_placement, stable=True)
    return new_to_old, ranks_sorted


def edge_renumbering(
    edge_indices: torch.Tensor,
    renumbered_nodes: torch.Tensor,
    vertex_mapping: torch.Tensor,
    edge_features: Optional[torch.Tensor] = None,
):
    """Relabel ``edge_indices[2, E]`` with ``old_to_new = inverse(renumbered_nodes)`` and
    sort edges by source rank (stable). ``vertex_mapping`` is the rank of each NEW id.
    Returns (edges[2,E], src_rank, dst_rank, edge_features)."""
    old_to_new = inverse_permutation(renumbered_nodes)
    src = old_to_new[edge_indices[0]]
    dst = old_to_new[edge_indices[1]]
    src_rank = vertex_mapping[src]
    dst_rank = vertex_mapping[dst]
    src_rank_sorted, order = torch.sort(src_rank, stable=True)
    src, dst, dst_rank = src[order], dst[order], dst_rank[order]
    if edge_features is not None:
        edge_features = edge_features[order]
    return torch.stack([src, dst], 0), src_rank_sorted, dst_rank, edge_features


def _to_tensor(a, dtype):
    if isinstance(a, torch.Tensor):
        return a.to(dtype)
    return torch.as_tensor(np.asarray(a)).to(dtype)


def process_homogenous_data(
    graph_data: dict,
    labels,
    rank: int,
    world_Size: int,
    split_idx: dict,
    node_rank_placement: torch.Tensor,
    *args,
    **kwargs,
) -> DistributedGraph:
    """OGB-style dict (``node_feat``, ``edge_index``, ``num_nodes``, ``edge_feat``) ->
    contiguous-ownership :class:`DistributedGraph` (features, labels and split index
    lists relabelled into the new numbering). Edge features are carried along."""
    for k in ("node_feat", "edge_index", "num_nodes"):
        if k not in graph_data:
            raise AssertionError(f"{k} not found")
    node_features = _to_tensor(graph_data["node_feat"], torch.float32)
    edge_index = _to_tensor(graph_data["edge_index"], torch.long)
    edge_feat = graph_data.get("edge_feat")
    edge_feat = None if edge_feat is None else _to_tensor(edge_feat, torch.float32)
    num_nodes = int(graph_data["num_nodes"])
    labels = _to_tensor(labels, torch.long).reshape(num_nodes, -1).squeeze(-1)
    if node_rank_placement.shape[0] != num_nodes:
        raise AssertionError("Node mapping mismatch")
    for k in ("train", "valid", "test"):
        if k not in split_idx:
            raise AssertionError(f"{k} split not found")
    new_to_old, ranks_of_new = node_renumbering(node_rank_placement.long())
    old_to_new = inverse_permutation(new_to_old)
    edge_index, src_rank, dst_rank, edge_feat = edge_renumbering(
        edge_index, new_to_old, ranks_of_new, edge_feat)
    split = {k: old_to_new[_to_tensor(split_idx[k], torch.long)] for k in ("train", "valid", "test")}
    return DistributedGraph(
        node_features=node_features[new_to_old],
        edge_index=edge_index,
        labels=labels[new_to_old],
        node_loc=ranks_of_new.long(),
        edge_loc=src_rank.long(),
        edge_dest_rank_mapping=dst_rank.long(),
        num_nodes=num_nodes,
        num_edges=int(edge_index.shape[1]),
        world_size=world_Size,
        edge_features=edge_feat,
        train_mask=split["train"],
        val_mask=split["valid"],
        test_mask=split["test"],
    )


def add_opposite_edges(edge_index: torch.Tensor) -> torch.Tensor:
    """Symmetrise a directed ``[2, E]`` edge list (OGB/preprocess.py:72-80)."""
    return torch.cat([edge_index, edge_index.flip(0)], dim=1)
