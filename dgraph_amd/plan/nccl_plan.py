"""Edge-centric gather/scatter plans (API generation G2).

Public surface of the reference's ``_NCCLCommPlan.py`` (``NCCLGraphCommPlan`` :10-100,
``NCCLEdgeConditionedGraphCommPlan`` :103-137, ``COO_to_NCCLCommPlan`` :174-278,
``COO_to_NCCLEdgeConditionedCommPlan`` :281-333); exact semantics in SURVEY.md App. C.2.

Differences by design:
* the boundary (rank, id) pairs are explicitly sorted (the reference relied on
  ``torch.unique(sorted=False)`` happening to sort, D10), and ids are not capped at 2^32;
* on first execution a plan is *lowered* (:meth:`NCCLGraphCommPlan.compiled`) to three
  static CSRs and a host-split all-to-all-v executor, so gather/scatter and both
  backwards are atomic-free segment sums with no host syncs.
"""
from __future__ import annotations

import sys
from dataclasses import dataclass, field, fields
from typing import Dict, List, Optional, Union

import torch
import torch.distributed as dist

from ..ops.csr import CSR
from .pattern import _alltoall_counts, _alltoallv_ids


@dataclass
class NCCLGraphCommPlan:
    rank: int
    world_size: int
    num_local_vertices: int
    num_local_edges: int
    local_edge_idx: torch.Tensor
    local_vertex_idx: torch.Tensor
    boundary_edge_idx: torch.Tensor
    boundary_edge_buffer_map: torch.Tensor
    boundary_edge_splits: List[int]
    boundary_vertex_idx: torch.Tensor
    boundary_vertex_splits: List[int]
    _compiled: Optional["CompiledPlan"] = field(default=None, repr=False, compare=False)

    def to(self, device: torch.device) -> "NCCLGraphCommPlan":
        self.local_edge_idx = self.local_edge_idx.to(device)
        self.local_vertex_idx = self.local_vertex_idx.to(device)
        self.boundary_edge_idx = self.boundary_edge_idx.to(device)
        self.boundary_edge_buffer_map = self.boundary_edge_buffer_map.to(device)
        self.boundary_vertex_idx = self.boundary_vertex_idx.to(device)
        self._compiled = None
        return self

    def memory_usage(self, unit: str = "MB") -> Dict[str, Union[float, str]]:
        div = {"B": 1, "KB": 1024, "MB": 1024**2, "GB": 1024**3}.get(unit.upper(), 1024**2)
        cpu = gpu = 0
        for f in fields(self):
            if f.name.startswith("_"):
                continue
            a = getattr(self, f.name)
            if isinstance(a, torch.Tensor):
                n = a.element_size() * a.nelement()
                if a.is_cuda:
                    gpu += n
                else:
                    cpu += n
            elif isinstance(a, list):
                cpu += sys.getsizeof(a) + sum(sys.getsizeof(i) for i in a)
            else:
                cpu += sys.getsizeof(a)
        return {"cpu": cpu / div, "gpu": gpu / div, "total": (cpu + gpu) / div,
                "unit": unit.upper()}

    def compiled(self, group=None) -> "CompiledPlan":
        if self._compiled is None:
            self._compiled = CompiledPlan.lower(self, group)
        return self._compiled

    def stats(self) -> dict:
        return {
            "rank": self.rank,
            "local_edges": int(self.local_edge_idx.numel()),
            "boundary_edges": int(self.boundary_edge_idx.numel()),
            "send_rows": int(sum(self.boundary_vertex_splits)),
            "recv_rows": int(sum(self.boundary_edge_splits)),
            "max_peer_send_rows": max(self.boundary_vertex_splits) if self.boundary_vertex_splits else 0,
        }


@dataclass
class NCCLEdgeConditionedGraphCommPlan:
    rank: int
    world_size: int
    source_graph_plan: NCCLGraphCommPlan
    dest_graph_plan: Optional[NCCLGraphCommPlan] = None

    def to(self, device: torch.device) -> "NCCLEdgeConditionedGraphCommPlan":
        self.source_graph_plan = self.source_graph_plan.to(device)
        if self.dest_graph_plan is not None:
            self.dest_graph_plan = self.dest_graph_plan.to(device)
        return self

    def reverse(self) -> "NCCLEdgeConditionedGraphCommPlan":
        if self.dest_graph_plan is None:
            raise ValueError("Destination graph plan is None, cannot reverse.")
        return NCCLEdgeConditionedGraphCommPlan(
            self.rank, self.world_size, self.dest_graph_plan, self.source_graph_plan
        )


class CompiledPlan:
    """Execution form of a :class:`NCCLGraphCommPlan`.

    * ``local``   CSR rows = local vertex, cols = local edge slot (vertex <- its edges)
    * ``pack``    CSR rows = send-buffer slot (unique (peer, id)), cols = boundary edge slot
    * ``unpack``  CSR rows = local vertex, cols = receive slot (requests of all peers)
    * ``a2a``     vertex-side -> edge-side all-to-all-v (reverse() for the other way)
    """

    def __init__(self, plan: NCCLGraphCommPlan, local: CSR, pack: CSR, unpack: CSR, a2a):
        self.plan = plan
        self.local = local
        self.pack = pack
        self.unpack = unpack
        self.a2a_v2e = a2a
        self.a2a_e2v = a2a.reversed()

    @staticmethod
    def lower(plan: NCCLGraphCommPlan, group=None) -> "CompiledPlan":
        from ..comm.alltoallv import AllToAllV

        N, E = plan.num_local_vertices, plan.num_local_edges
        local = CSR.from_coo(plan.local_vertex_idx.long(), plan.local_edge_idx.long(), N, E,
                             keep_perm=False)
        nbuf = int(sum(plan.boundary_edge_splits))
        pack = CSR.from_coo(plan.boundary_edge_buffer_map.long(), plan.boundary_edge_idx.long(),
                            nbuf, E, keep_perm=False)
        nrecv = plan.boundary_vertex_idx.numel()
        unpack = CSR.from_coo(plan.boundary_vertex_idx.long(),
                              torch.arange(nrecv, device=plan.boundary_vertex_idx.device),
                              N, nrecv, keep_perm=False)
        a2a = AllToAllV(plan.boundary_vertex_splits, plan.boundary_edge_splits, group)
        return CompiledPlan(plan, local, pack, unpack, a2a)


def compute_edge_slices(dest_ranks, rank, my_dst_global, offset):
    """Split local edges into rank-internal and boundary ones (reference helper)."""
    internal = dest_ranks == rank
    internal_node_idx = my_dst_global[internal] - offset[rank]
    internal_edge_indices = torch.nonzero(internal, as_tuple=True)[0]
    remote = ~internal
    boundary_edge_indices = torch.nonzero(remote, as_tuple=True)[0]
    return (internal_node_idx, internal_edge_indices, my_dst_global[remote],
            dest_ranks[remote], boundary_edge_indices)


def fast_2D_unique(indices_1: torch.Tensor, indices_2: torch.Tensor):
    """Unique (a, b) pairs, explicitly sorted by (a, b) (D10), with the inverse map."""
    a = indices_1.long()
    b = indices_2.long()
    span = int(b.max().item()) + 1 if b.numel() else 1
    key = a * span + b
    uniq, inverse = torch.unique(key, sorted=True, return_inverse=True)
    ua = torch.div(uniq, span, rounding_mode="floor")
    return ua, uniq - ua * span, inverse


def COO_to_NCCLCommPlan(
    rank: int,
    world_size: int,
    global_edges_vertex_ids: Optional[torch.Tensor] = None,
    local_edge_list: Optional[torch.Tensor] = None,
    offset: Optional[torch.Tensor] = None,
    group: Optional[dist.ProcessGroup] = None,
    **legacy_kwargs,
) -> NCCLGraphCommPlan:
    """Collective plan build for the vertex ids referenced by this rank's edges.

    ``offset[W+1]``: rank r owns global ids ``[offset[r], offset[r+1])`` (I1).
    ``local_edge_list``: indices (into ``global_edges_vertex_ids``) of this rank's edges.
    (``global_edges_dst=`` is accepted as an alias, the name the reference's own test
    used, D6.)
    """
    if global_edges_vertex_ids is None and "global_edges_dst" in legacy_kwargs:
        global_edges_vertex_ids = legacy_kwargs.pop("global_edges_dst")
    device = local_edge_list.device
    offset = offset.to(device).long()
    my_ids = global_edges_vertex_ids.to(device)[local_edge_list].long()
    my_start = int(offset[rank])
    my_end = int(offset[rank + 1])
    dest_ranks = torch.bucketize(my_ids, offset, right=True) - 1
    (internal_node_idx, internal_edge_idx, b_ids, b_ranks, boundary_edge_idx) = \
        compute_edge_slices(dest_ranks, rank, my_ids, offset)
    u_rank, u_ids, inverse = fast_2D_unique(b_ranks, b_ids)
    edge_splits_t = torch.bincount(u_rank, minlength=world_size) if u_rank.numel() else \
        torch.zeros(world_size, dtype=torch.long, device=device)
    edge_splits = [int(v) for v in edge_splits_t.tolist()]
    if world_size > 1 and dist.is_initialized():
        vertex_splits_t = _alltoall_counts(edge_splits_t, group)
        vertex_splits = [int(v) for v in vertex_splits_t.tolist()]
        recv_ids = _alltoallv_ids(u_ids, edge_splits, vertex_splits, group)
    else:
        vertex_splits = [0] * world_size
        recv_ids = u_ids[:0]
    return NCCLGraphCommPlan(
        rank=rank,
        world_size=world_size,
        num_local_vertices=my_end - my_start,
        num_local_edges=int(local_edge_list.numel()),
        local_edge_idx=internal_edge_idx,
        local_vertex_idx=internal_node_idx,
        boundary_edge_idx=boundary_edge_idx,
        boundary_edge_buffer_map=inverse,
        boundary_edge_splits=edge_splits,
        boundary_vertex_idx=(recv_ids - my_start).to(device),
        boundary_vertex_splits=vertex_splits,
    )


def COO_to_NCCLEdgeConditionedCommPlan(
    rank: int,
    world_size: int,
    global_edges_src: torch.Tensor,
    global_edges_dst: torch.Tensor,
    local_edge_list: torch.Tensor,
    src_offset: torch.Tensor,
    dest_offset: Optional[torch.Tensor] = None,
    group: Optional[dist.ProcessGroup] = None,
) -> NCCLEdgeConditionedGraphCommPlan:
    src_plan = COO_to_NCCLCommPlan(rank, world_size, global_edges_src, local_edge_list,
                                   src_offset, group)
    dst_plan = COO_to_NCCLCommPlan(rank, world_size, global_edges_dst, local_edge_list,
                                   src_offset if dest_offset is None else dest_offset, group)
    return NCCLEdgeConditionedGraphCommPlan(rank, world_size, src_plan, dst_plan)
