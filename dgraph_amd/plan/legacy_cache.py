"""Static precomputes for the index-based API (G1): ``NCCLGatherCache`` /
``NCCLScatterCache`` and their generators, plus the reference's index helpers.

Reference: DGraph/distributed/nccl/_nccl_cache.py:16-312 and _indices_utils.py:5-245.
There, a cache was a bag of per-peer masks/placement dicts consumed by a legacy code
path that could not run (D1). Here a cache *is* a lowered
:class:`~dgraph_amd.plan.nccl_plan.NCCLGraphCommPlan` (plus the legacy scalar fields that
scripts read), produced WITHOUT communication: in the global index form every rank sees
every edge's placement and owner, so rank ``r``'s plan — including what its peers will
request from it — is a pure function of the index arrays. This is what lets caches be
generated offline for any (rank, world_size) from one process, as the reference's
OGB-LSC/CacheGenerator.py:119-170 did with a dummy communicator.

``comm.gather(x, indices, rank_mappings, cache=...)`` /
``comm.scatter(..., cache=...)`` execute a cache directly.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from .nccl_plan import NCCLGraphCommPlan, fast_2D_unique


def lower_global_form_offline(
    indices: torch.Tensor,
    edge_placement: torch.Tensor,
    edge_dest_ranks: torch.Tensor,
    rows_per_rank: List[int],
    rank: int,
    world_size: int,
) -> NCCLGraphCommPlan:
    """Plan of ``rank`` for edges ``e`` placed on ``edge_placement[e]`` that reference
    vertex ``indices[e]`` (local row ``indices[e] mod rows_per_rank[owner]``) owned by
    ``edge_dest_ranks[e]`` — computed locally, no collectives."""
    idx = indices.reshape(-1).long()
    place = edge_placement.reshape(-1).long().to(idx.device)
    own = edge_dest_ranks.reshape(-1).long().to(idx.device)
    rows = torch.tensor(rows_per_rank, dtype=torch.long, device=idx.device)
    local_row = torch.remainder(idx, rows[own].clamp(min=1))

    def side(r: int):
        """(edge ids placed on r, owner, local row) with (owner, row)-sorted uniques."""
        e = torch.nonzero(place == r, as_tuple=True)[0]
        o, lr = own[e], local_row[e]
        remote = o != r
        uo, ur, inv = fast_2D_unique(o[remote], lr[remote])
        return e, o, lr, remote, uo, ur, inv

    e, o, lr, remote, uo, ur, inv = side(rank)
    internal = ~remote
    edge_splits = torch.bincount(uo, minlength=world_size).tolist() if uo.numel() else [0] * world_size
    # what every peer p requests from me, in p's (owner, row) order -> my send list
    vertex_idx, vertex_splits = [], []
    for p in range(world_size):
        if p == rank:
            vertex_splits.append(0)
            continue
        _, _, _, _, puo, pur, _ = side(p)
        mine = pur[puo == rank]
        vertex_idx.append(mine)
        vertex_splits.append(int(mine.numel()))
    vidx = torch.cat(vertex_idx) if vertex_idx else idx.new_zeros(0)
    return NCCLGraphCommPlan(
        rank=rank,
        world_size=world_size,
        num_local_vertices=int(rows_per_rank[rank]),
        num_local_edges=int(e.numel()),
        local_edge_idx=torch.nonzero(internal, as_tuple=True)[0],
        local_vertex_idx=lr[internal],
        boundary_edge_idx=torch.nonzero(remote, as_tuple=True)[0],
        boundary_edge_buffer_map=inv,
        boundary_edge_splits=[int(v) for v in edge_splits],
        boundary_vertex_idx=vidx,
        boundary_vertex_splits=vertex_splits,
    )


@dataclass
class NCCLGatherCache:
    """Precomputed vertex->edge gather for the G1 global index form."""

    plan: NCCLGraphCommPlan
    rank: int
    world_size: int
    gather_num_output_rows: int
    gather_needs_comm: bool

    @property
    def scatter_num_remote_rows(self) -> int:  # backward (scatter) side
        return int(sum(self.plan.boundary_edge_splits))

    def to(self, device):
        self.plan = self.plan.to(device)
        return self


@dataclass
class NCCLScatterCache:
    """Precomputed edge->vertex scatter-sum for the G1 global index form."""

    plan: NCCLGraphCommPlan
    rank: int
    world_size: int
    scatter_num_remote_rows: int
    gather_num_output_rows: int

    def to(self, device):
        self.plan = self.plan.to(device)
        return self


def NCCLGatherCacheGenerator(indices, edge_placement, edge_dest_ranks, num_input_rows: int,
                             rank: int, world_size: int,
                             rows_per_rank: Optional[List[int]] = None) -> NCCLGatherCache:
    rows = rows_per_rank or [int(num_input_rows)] * world_size
    plan = lower_global_form_offline(indices, edge_placement, edge_dest_ranks, rows, rank,
                                     world_size)
    return NCCLGatherCache(plan, rank, world_size, plan.num_local_edges,
                           plan.boundary_edge_idx.numel() > 0 or sum(plan.boundary_vertex_splits) > 0)


def NCCLScatterCacheGenerator(indices, edge_placement, edge_dest_ranks, num_output_rows: int,
                              rank: int, world_size: int,
                              rows_per_rank: Optional[List[int]] = None) -> NCCLScatterCache:
    rows = rows_per_rank or [int(num_output_rows)] * world_size
    plan = lower_global_form_offline(indices, edge_placement, edge_dest_ranks, rows, rank,
                                     world_size)
    return NCCLScatterCache(plan, rank, world_size, int(sum(plan.boundary_vertex_splits)),
                            plan.num_local_edges)


def save_cache(cache, path: str) -> None:
    """Plain-tensor serialisation (loads with ``weights_only=True``)."""
    p = cache.plan
    torch.save({"kind": type(cache).__name__, "rank": cache.rank, "world_size": cache.world_size,
                "num_local_vertices": p.num_local_vertices, "num_local_edges": p.num_local_edges,
                "local_edge_idx": p.local_edge_idx, "local_vertex_idx": p.local_vertex_idx,
                "boundary_edge_idx": p.boundary_edge_idx,
                "boundary_edge_buffer_map": p.boundary_edge_buffer_map,
                "boundary_edge_splits": torch.tensor(p.boundary_edge_splits),
                "boundary_vertex_idx": p.boundary_vertex_idx,
                "boundary_vertex_splits": torch.tensor(p.boundary_vertex_splits)}, path)


def load_cache(path: str, map_location="cpu"):
    d = torch.load(path, map_location=map_location, weights_only=True)
    plan = NCCLGraphCommPlan(
        d["rank"], d["world_size"], d["num_local_vertices"], d["num_local_edges"],
        d["local_edge_idx"], d["local_vertex_idx"], d["boundary_edge_idx"],
        d["boundary_edge_buffer_map"], d["boundary_edge_splits"].tolist(),
        d["boundary_vertex_idx"], d["boundary_vertex_splits"].tolist())
    if d["kind"] == "NCCLGatherCache":
        return NCCLGatherCache(plan, d["rank"], d["world_size"], plan.num_local_edges,
                               True)
    return NCCLScatterCache(plan, d["rank"], d["world_size"],
                            int(sum(plan.boundary_vertex_splits)), plan.num_local_edges)


# ---------------------------------------------------------------------------------------
# Index helpers (reference _indices_utils.py), vectorised
# ---------------------------------------------------------------------------------------
def _get_send_comm_vector(comm_senders, comm_receivers, rank: int, world_size: int):
    return torch.bincount(comm_receivers[comm_senders == rank], minlength=world_size).long()


def _get_recv_comm_vector(comm_senders, comm_receivers, rank: int, world_size: int):
    return torch.bincount(comm_senders[comm_receivers == rank], minlength=world_size).long()


def _get_send_recv_comm_vectors(src_ranks, dest_ranks, rank: int, world_size: int):
    m = src_ranks != dest_ranks
    s, r = src_ranks[m], dest_ranks[m]
    return (_get_send_comm_vector(s, r, rank, world_size),
            _get_recv_comm_vector(s, r, rank, world_size))


def _get_local_send_placement(send_comm_vector, indices, src_ranks, dest_ranks, rank: int,
                              num_src_rows: int) -> Dict[int, torch.Tensor]:
    out = {}
    idx = indices.reshape(-1)
    for i, n in enumerate(send_comm_vector.tolist()):
        if n == 0 or i == rank:
            continue
        m = (src_ranks == rank) & (dest_ranks == i)
        out[i] = idx[m] % num_src_rows
    return out


def _generate_local_rank_mapping(_global_rank_mapping: torch.Tensor, world_size: int) -> torch.Tensor:
    """Equal contiguous blocks of ranks over the flattened mapping (last block may be short)."""
    n = _global_rank_mapping.numel()
    per = (n + world_size - 1) // world_size
    return (torch.arange(n) // max(per, 1)).long()
