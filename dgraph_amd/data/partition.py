"""Vertex partitioners and partition statistics.

The reference relied on external METIS runs (experiments/OGB/preprocess.py:15-47 via
networkx + metis; neither is installed here). This module provides in-library
partitioners that run on device tensors:

* ``contiguous``   — equal id blocks (what synthetic/locality-ordered graphs want);
* ``round_robin``  — ``i mod W`` (the reference's fallback);
* ``random``       — seeded uniform;
* ``label_propagation`` — balanced label propagation refining an initial partition:
  each round every vertex picks the most frequent partition among its neighbours
  (vectorised bincount over (vertex, part) pairs), moves are admitted in random order
  only while the target part stays under ``(1 + imbalance) * V / W``;
* ``metis``        — used only if a ``metis`` Python binding is importable.

:func:`partition_stats` reports the edge cut and the per-pair halo volume; the MAX pair
volume is what bounds an all-to-all-v over point-to-point xGMI links (§5.8).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch


def contiguous_partition(num_nodes: int, world_size: int, device="cpu") -> torch.Tensor:
    base, rem = divmod(num_nodes, world_size)
    sizes = torch.full((world_size,), base, dtype=torch.long)
    sizes[:rem] += 1
    return torch.repeat_interleave(torch.arange(world_size), sizes).to(device)


def round_robin_partition(num_nodes: int, world_size: int, device="cpu") -> torch.Tensor:
    return torch.arange(num_nodes, device=device) % world_size


def random_partition(num_nodes: int, world_size: int, seed: int = 0, device="cpu") -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, world_size, (num_nodes,), generator=g).to(device)


def label_propagation_partition(
    edge_index: torch.Tensor,
    num_nodes: int,
    world_size: int,
    rounds: int = 10,
    imbalance: float = 0.05,
    init: Optional[torch.Tensor] = None,
    seed: int = 0,
) -> torch.Tensor:
    """Balanced label propagation over an undirected view of ``edge_index[2, E]``."""
    dev = edge_index.device
    part = (init.clone() if init is not None else contiguous_partition(num_nodes, world_size, dev)).long()
    src = torch.cat([edge_index[0], edge_index[1]]).long()
    dst = torch.cat([edge_index[1], edge_index[0]]).long()
    cap = int((1.0 + imbalance) * num_nodes / world_size) + 1
    g = torch.Generator(device="cpu").manual_seed(seed)
    for _ in range(rounds):
        # neighbour-part histogram per vertex: counts[v, p]
        key = src * world_size + part[dst]
        counts = torch.bincount(key, minlength=num_nodes * world_size).view(num_nodes, world_size)
        best = counts.argmax(1)
        gain = counts.gather(1, best[:, None]).squeeze(1) - counts.gather(1, part[:, None]).squeeze(1)
        cand = torch.nonzero((best != part) & (gain > 0), as_tuple=True)[0]
        if cand.numel() == 0:
            break
        cand = cand[torch.randperm(cand.numel(), generator=g).to(dev)]
        sizes = torch.bincount(part, minlength=world_size)
        # admit moves per target part up to its remaining capacity (sequential within a
        # round in random order, vectorised by ranking candidates per target part)
        tgt = best[cand]
        order = torch.argsort(tgt, stable=True)
        cand, tgt = cand[order], tgt[order]
        first = torch.searchsorted(tgt, torch.arange(world_size, device=dev))
        rank_in_tgt = torch.arange(cand.numel(), device=dev) - first[tgt]
        room = (cap - sizes).clamp(min=0)
        ok = rank_in_tgt < room[tgt]
        moved = cand[ok]
        if moved.numel() == 0:
            break
        part[moved] = tgt[ok]
    return part


def metis_partition(edge_index: torch.Tensor, num_nodes: int, world_size: int) -> torch.Tensor:
    import metis  # type: ignore  # optional

    adj = [[] for _ in range(num_nodes)]
    for s, d in edge_index.t().tolist():
        if s != d:
            adj[s].append(d)
            adj[d].append(s)
    _, parts = metis.part_graph(adj, world_size)
    return torch.tensor(parts, dtype=torch.long)


def partition(method: str, num_nodes: int, world_size: int,
              edge_index: Optional[torch.Tensor] = None, **kw) -> torch.Tensor:
    if method == "contiguous":
        return contiguous_partition(num_nodes, world_size)
    if method in ("round_robin", "round-robin"):
        return round_robin_partition(num_nodes, world_size)
    if method == "random":
        return random_partition(num_nodes, world_size, **kw)
    if method in ("label_propagation", "lp"):
        return label_propagation_partition(edge_index, num_nodes, world_size, **kw)
    if method == "metis":
        return metis_partition(edge_index, num_nodes, world_size)
    raise ValueError(f"unknown partition method {method}")


def partition_stats(edge_index: torch.Tensor, part: torch.Tensor, world_size: int) -> Dict:
    """Edge cut and halo volume per (owner -> requester) pair, for edges (central=src,
    neighbour=dst): rank ``part[src]`` needs ``dst`` from ``part[dst]``."""
    src, dst = edge_index[0].long(), edge_index[1].long()
    ps, pd = part[src], part[dst]
    cut = ps != pd
    n_nodes = part.numel()
    # unique (requester, vertex) pairs
    key = torch.unique(ps[cut] * n_nodes + dst[cut])
    req = torch.div(key, n_nodes, rounding_mode="floor")
    own = part[key - req * n_nodes]
    pair = torch.bincount(own * world_size + req, minlength=world_size * world_size)
    pair = pair.view(world_size, world_size)
    sizes = torch.bincount(part, minlength=world_size)
    return {
        "edge_cut_frac": float(cut.float().mean()) if cut.numel() else 0.0,
        "halo_rows_total": int(pair.sum()),
        "halo_rows_max_pair": int(pair.max()) if pair.numel() else 0,
        "halo_rows_per_rank_max": int(pair.sum(0).max()) if pair.numel() else 0,
        "imbalance": float(sizes.max() / max(sizes.float().mean(), 1.0)),
        "pair_matrix": pair,
    }
