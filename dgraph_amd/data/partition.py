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


def _admit_moves(cand, best, sizes, cap, world_size, g, dev):
    """Random-order admission of candidate moves per target part under the size cap."""
    cand = cand[torch.randperm(cand.numel(), generator=g).to(dev)]
    tgt = best[cand]
    order = torch.argsort(tgt, stable=True)
    cand, tgt = cand[order], tgt[order]
    first = torch.searchsorted(tgt, torch.arange(world_size, device=dev))
    rank_in_tgt = torch.arange(cand.numel(), device=dev) - first[tgt]
    room = (cap - sizes).clamp(min=0)
    ok = rank_in_tgt < room[tgt]
    return cand[ok], tgt[ok]


_LP_CHUNK = 1 << 28  # edges per histogram step (bounded temporaries at 1e9+ edges)


def _neighbour_part_counts(rows, cols, part, n_rows, world_size, counts=None):
    """counts[v, p] += #{edges (v, u) : part[u] == p}, chunked over the edge list."""
    if counts is None:
        counts = torch.zeros(n_rows * world_size, dtype=torch.int64, device=rows.device)
    else:
        counts = counts.view(-1)
    for a in range(0, rows.numel(), _LP_CHUNK):
        key = rows[a:a + _LP_CHUNK].long() * world_size + part[cols[a:a + _LP_CHUNK].long()]
        counts += torch.bincount(key, minlength=n_rows * world_size)
        del key
    return counts.view(n_rows, world_size)


def label_propagation_partition(
    edge_index: torch.Tensor,
    num_nodes: int,
    world_size: int,
    rounds: int = 10,
    imbalance: float = 0.05,
    init: Optional[torch.Tensor] = None,
    seed: int = 0,
) -> torch.Tensor:
    """Balanced label propagation over an undirected view of ``edge_index[2, E]``.

    Each round every vertex counts its neighbours per part (two chunked bincount passes,
    one per edge direction: no 2E concatenation, so a 1.6e9-edge papers100M graph fits one
    GPU), picks the most frequent part, and moves with positive gain are admitted in random
    order while the target stays under ``(1 + imbalance) * V / W``."""
    dev = edge_index.device
    part = (init.clone() if init is not None else contiguous_partition(num_nodes, world_size, dev)).long()
    cap = int((1.0 + imbalance) * num_nodes / world_size) + 1
    g = torch.Generator(device="cpu").manual_seed(seed)
    for _ in range(rounds):
        counts = _neighbour_part_counts(edge_index[0], edge_index[1], part, num_nodes, world_size)
        counts = _neighbour_part_counts(edge_index[1], edge_index[0], part, num_nodes, world_size,
                                        counts)
        best = counts.argmax(1)
        gain = counts.gather(1, best[:, None]).squeeze(1) - counts.gather(1, part[:, None]).squeeze(1)
        del counts
        cand = torch.nonzero((best != part) & (gain > 0), as_tuple=True)[0]
        if cand.numel() == 0:
            break
        sizes = torch.bincount(part, minlength=world_size)
        moved, tgt = _admit_moves(cand, best, sizes, cap, world_size, g, dev)
        if moved.numel() == 0:
            break
        part[moved] = tgt
    return part


def distributed_label_propagation(
    rowptr: torch.Tensor,
    col: torch.Tensor,
    lo: int,
    num_nodes: int,
    world_size: int,
    group=None,
    rounds: int = 10,
    imbalance: float = 0.05,
    init: Optional[torch.Tensor] = None,
    seed: int = 0,
) -> torch.Tensor:
    """Label propagation where every rank holds only its own rows' adjacency.

    ``rowptr/col`` is the CSR of rows ``[lo, lo + L)`` with GLOBAL column ids and both edge
    directions (the symmetrised aggregation CSR every trainer builds anyway). The part
    vector (one int64 per vertex) is replicated. Per round each rank histograms its rows'
    neighbour parts, proposes its positive-gain moves, and receives a share of every target
    part's remaining room proportional to its proposals (one all-reduce of W counts, so the
    shares never over-fill a part); the admitted moves of all ranks are all-gathered and
    applied identically everywhere. Collective over ``group``; returns the replicated
    part vector."""
    import torch.distributed as dist

    dev = col.device
    L = rowptr.numel() - 1
    part = (init.clone() if init is not None else contiguous_partition(num_nodes, world_size, dev)).long().to(dev)
    cap = int((1.0 + imbalance) * num_nodes / world_size) + 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    nranks = dist.get_world_size(group) if dist.is_initialized() else 1
    g = torch.Generator(device="cpu").manual_seed(seed * 1_000_003 + rank)
    rows = torch.repeat_interleave(torch.arange(L, device=dev), rowptr[1:] - rowptr[:-1])
    mine = torch.arange(lo, lo + L, device=dev)
    for _ in range(rounds):
        counts = _neighbour_part_counts(rows, col, part, L, world_size)
        cur = part[mine]
        best = counts.argmax(1)
        gain = counts.gather(1, best[:, None]).squeeze(1) - counts.gather(1, cur[:, None]).squeeze(1)
        del counts
        cand = torch.nonzero((best != cur) & (gain > 0), as_tuple=True)[0]
        prop = torch.bincount(best[cand], minlength=world_size)
        tot = prop.clone()
        if nranks > 1:
            dist.all_reduce(tot, group=group)
        if int(tot.sum()) == 0:
            break
        sizes = torch.bincount(part, minlength=world_size)
        room = (cap - sizes).clamp(min=0)
        share = torch.where(tot > 0, room * prop // tot.clamp(min=1), torch.zeros_like(room))
        moved, tgt = _admit_moves(cand, best, cap - share, cap, world_size, g, dev)
        moved = moved + lo
        if nranks > 1:
            n = torch.tensor([moved.numel()], device=dev)
            ns = [torch.zeros_like(n) for _ in range(nranks)]
            dist.all_gather(ns, n, group=group)
            m = max(int(v) for v in ns)
            pay = torch.full((2, m), -1, dtype=torch.long, device=dev)
            pay[0, :moved.numel()] = moved
            pay[1, :moved.numel()] = tgt
            got = [torch.empty_like(pay) for _ in range(nranks)]
            dist.all_gather(got, pay, group=group)
            allp = torch.cat(got, 1)
            allp = allp[:, allp[0] >= 0]
            moved, tgt = allp[0], allp[1]
        if moved.numel() == 0:
            break
        part[moved] = tgt
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


def partition_stats(edge_index: torch.Tensor, part: torch.Tensor, world_size: int,
                    symmetric: bool = False) -> Dict:
    """Edge cut and halo volume per (owner -> requester) pair, for edges (central=src,
    neighbour=dst): rank ``part[src]`` needs ``dst`` from ``part[dst]``. With
    ``symmetric`` every edge also runs dst -> src (messages both ways, as in the
    symmetrised aggregation); the edge list is processed in chunks either way."""
    n_nodes = part.numel()
    # needed[q, v]: requester q must receive vertex v (a W x V byte map instead of a sort
    # of (requester, vertex) keys: 0.9 GB at W = 8 on papers100M, no 2^31-element unique)
    needed = torch.zeros(world_size * n_nodes, dtype=torch.bool, device=part.device)
    n_cut = n_all = 0
    dirs = ((0, 1), (1, 0)) if symmetric else ((0, 1),)
    for a in range(0, edge_index.shape[1], _LP_CHUNK):
        for i, j in dirs:
            src = edge_index[i, a:a + _LP_CHUNK].long()
            dst = edge_index[j, a:a + _LP_CHUNK].long()
            ps = part[src]
            cut = ps != part[dst]
            n_cut += int(cut.sum())
            n_all += int(cut.numel())
            needed[ps[cut] * n_nodes + dst[cut]] = True
            del src, dst, ps, cut
    needed = needed.view(world_size, n_nodes)
    pair = torch.stack([torch.bincount(part[needed[q]], minlength=world_size)
                        for q in range(world_size)], 1)  # [owner, requester]
    del needed
    sizes = torch.bincount(part, minlength=world_size)
    return {
        "edge_cut_frac": n_cut / n_all if n_all else 0.0,
        "halo_rows_total": int(pair.sum()),
        "halo_rows_max_pair": int(pair.max()) if pair.numel() else 0,
        "halo_rows_per_rank_max": int(pair.sum(0).max()) if pair.numel() else 0,
        "imbalance": float(sizes.max() / max(sizes.float().mean(), 1.0)),
        "pair_matrix": pair,
    }
