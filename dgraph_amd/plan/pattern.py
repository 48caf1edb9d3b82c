"""Vertex-centric halo communication pattern (API generation G3).

Public surface of the reference's ``DGraph/distributed/commInfo.py`` (dataclass
``CommunicationPattern`` :7-32 and the ``compute_*`` helpers :35-164), re-implemented:

* the ``compute_*`` helpers keep the reference's literal semantics (they are what
  tests/test_comm_info.py pins down);
* :func:`build_communication_pattern` is *request based*: every rank announces the halo
  rows it needs to their owners with one all-to-all, so the receive layout is
  ``(owner rank, global id)``-sorted by construction and correct for ANY partition and
  for non-symmetric or bipartite edge sets (the reference is only correct for symmetric
  graphs under contiguous ownership, invariant I3 / Appendix C.1). On symmetric graphs
  the result is identical to the reference's.
* it accepts ``neighbor_partitioning=`` for bipartite relations (the call made by the
  reference's GraphCast code, graphcast_graph.py:110-153, that its builder rejects: D5).

Edge lists are ``[E, 2]`` of ``(central, neighbor)`` global ids: the central (column 0)
vertex aggregates, the neighbor (column 1) vertex's features are exchanged.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


@dataclass
class CommunicationPattern:
    # --- Identity ---
    rank: int
    world_size: int
    # --- Vertex counts ---
    num_local_vertices: int
    num_halo_vertices: int
    # --- Local subgraph: [E_local, 2] in local numbering; col 1 in [0, L_nbr + H) ---
    local_edge_list: torch.Tensor
    # --- Send indexing (rows of the local neighbour-feature matrix) ---
    send_local_idx: torch.Tensor
    send_offset: torch.Tensor
    # --- Receive indexing ---
    recv_offset: torch.Tensor
    # --- comm_map[q, p] = rows rank q sends to rank p (int64) ---
    comm_map: torch.Tensor
    # --- One-sided write offsets (Appendix C.1) ---
    put_forward_remote_offset: torch.Tensor
    put_backward_remote_offset: torch.Tensor
    # --- dgraph_amd extensions (not in the reference dataclass) ---
    halo_vertices: Optional[torch.Tensor] = None      # global ids, receive order
    local_vertices: Optional[torch.Tensor] = None     # global ids of local centrals
    num_local_neighbor_vertices: Optional[int] = None  # L_nbr (== L when homogeneous)
    _cache: dict = field(default_factory=dict, repr=False)

    # Host-side split lists, computed once (no per-exchange .tolist()).
    def send_splits(self) -> List[int]:
        if "send_splits" not in self._cache:
            o = self.send_offset.detach().cpu().tolist()
            self._cache["send_splits"] = [int(o[i + 1] - o[i]) for i in range(len(o) - 1)]
        return self._cache["send_splits"]

    def recv_splits(self) -> List[int]:
        if "recv_splits" not in self._cache:
            o = self.recv_offset.detach().cpu().tolist()
            self._cache["recv_splits"] = [int(o[i + 1] - o[i]) for i in range(len(o) - 1)]
        return self._cache["recv_splits"]

    def to(self, device) -> "CommunicationPattern":
        for name in ("local_edge_list", "send_local_idx", "halo_vertices", "local_vertices"):
            t = getattr(self, name)
            if isinstance(t, torch.Tensor):
                setattr(self, name, t.to(device))
        self._cache.pop("send_map", None)
        return self

    def stats(self) -> dict:
        """Plan statistics: halo rows per peer (max pairwise volume is what bounds an
        all-to-all-v over point-to-point xGMI links)."""
        cm = self.comm_map.detach().cpu()
        off = cm.clone()
        off.fill_diagonal_(0)
        return {
            "rank": self.rank,
            "world_size": self.world_size,
            "num_local": self.num_local_vertices,
            "num_halo": self.num_halo_vertices,
            "num_local_edges": int(self.local_edge_list.shape[0]),
            "send_rows": int(self.send_offset[-1]),
            "recv_rows": int(self.recv_offset[-1]),
            "max_pair_rows": int(off.max()) if off.numel() else 0,
            "total_rows": int(off.sum()),
        }


# --------------------------------------------------------------------------------------
# Reference-compatible helpers (literal semantics of commInfo.py:35-164)
# --------------------------------------------------------------------------------------
def compute_local_vertices(partitioning: torch.Tensor, rank: int) -> torch.Tensor:
    """Global ids owned by ``rank`` (ascending)."""
    return torch.nonzero(partitioning == rank, as_tuple=True)[0]


def compute_halo_vertices(
    edge_list: torch.Tensor,
    src_partitioning: torch.Tensor,
    rank: int,
    dst_partitioning: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """Sorted unique column-1 ids of edges whose column-0 vertex is local and whose
    column-1 vertex is remote."""
    dst_partitioning = src_partitioning if dst_partitioning is None else dst_partitioning
    cross = (src_partitioning[edge_list[:, 0]] == rank) & (dst_partitioning[edge_list[:, 1]] != rank)
    return torch.unique(edge_list[cross, 1])


def _inverse_map(ids: torch.Tensor, size: int, base: int = 0) -> torch.Tensor:
    inv = torch.full((size,), -1, dtype=torch.long, device=ids.device)
    inv[ids] = torch.arange(base, base + ids.numel(), device=ids.device)
    return inv


def compute_local_edge_list(
    global_edge_list: torch.Tensor,
    partitioning: torch.Tensor,
    local_vertices_global: torch.Tensor,
    halo_vertices_global: torch.Tensor,
    rank: int,
) -> torch.Tensor:
    """Edges with a local column-0 vertex, renumbered: local -> [0, L), halo -> [L, L+H)."""
    n = partitioning.numel()
    g2l = _inverse_map(local_vertices_global, n)
    g2l[halo_vertices_global] = torch.arange(
        local_vertices_global.numel(),
        local_vertices_global.numel() + halo_vertices_global.numel(),
        device=g2l.device,
    )
    mine = global_edge_list[partitioning[global_edge_list[:, 0]] == rank]
    return g2l[mine]


def compute_boundary_vertices(
    edge_list: torch.Tensor,
    src_partitioning: torch.Tensor,
    src_local_vertices_global: torch.Tensor,
    rank: int,
    num_ranks: int,
    dst_partitioning: Optional[torch.Tensor] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Local column-0 vertices with an edge to each remote rank (deduplicated per
    destination rank, grouped by rank ascending, ids ascending) and their CSR offsets."""
    dst_partitioning = src_partitioning if dst_partitioning is None else dst_partitioning
    src_rank = src_partitioning[edge_list[:, 0]]
    dst_rank = dst_partitioning[edge_list[:, 1]]
    cross = (src_rank == rank) & (dst_rank != rank)
    src = edge_list[cross, 0]
    tgt = dst_rank[cross]
    nsrc = src_partitioning.numel()
    key = torch.unique(tgt * nsrc + src)  # sorted: by target rank, then id (I5)
    tgt_u = torch.div(key, nsrc, rounding_mode="floor")
    src_u = key - tgt_u * nsrc
    g2l = _inverse_map(src_local_vertices_global, nsrc)
    send_local_idx = g2l[src_u]
    counts = torch.bincount(tgt_u, minlength=num_ranks) if tgt_u.numel() else \
        torch.zeros(num_ranks, dtype=torch.long, device=edge_list.device)
    send_offset = torch.zeros(num_ranks + 1, dtype=torch.long, device=edge_list.device)
    send_offset[1:] = torch.cumsum(counts, 0)
    return send_local_idx, send_offset


def _comm_device(ref: torch.Tensor, group=None) -> torch.device:
    from ..comm.groups import comm_device

    return comm_device(group)


def compute_comm_map(send_offset: torch.Tensor, world_size: int,
                     group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """All-gather of per-peer send counts -> ``comm_map[W, W]`` (int64; D11)."""
    counts = (send_offset[1:] - send_offset[:-1]).long()
    if not dist.is_initialized() or world_size == 1:
        return counts.view(1, -1).clone()
    dev = _comm_device(counts, group)
    parts = [torch.zeros(world_size, dtype=torch.long, device=dev) for _ in range(world_size)]
    dist.all_gather(parts, counts.to(dev), group=group)
    return torch.stack(parts).to(send_offset.device)


def compute_recv_offsets(comm_map: torch.Tensor, rank: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(recv_offset[W+1] on CPU, one-sided backward write offsets ``comm_map[:rank].sum(0)``)."""
    recv = comm_map[:, rank].detach().cpu().long()
    recv_offset = torch.zeros(comm_map.shape[0] + 1, dtype=torch.long)
    recv_offset[1:] = torch.cumsum(recv, 0)
    return recv_offset, comm_map[:rank, :].sum(0)


# --------------------------------------------------------------------------------------
# Request-based builder
# --------------------------------------------------------------------------------------
def _alltoall_counts(counts: torch.Tensor, group=None) -> torch.Tensor:
    dev = _comm_device(counts, group)
    out = torch.empty_like(counts, device=dev)
    dist.all_to_all_single(out, counts.to(dev), group=group)
    return out.to(counts.device)


def _alltoallv_ids(ids: torch.Tensor, send_splits: List[int], recv_splits: List[int],
                   group=None) -> torch.Tensor:
    dev = _comm_device(ids, group)
    out = torch.empty(sum(recv_splits), dtype=ids.dtype, device=dev)
    dist.all_to_all_single(out, ids.to(dev).contiguous(), output_split_sizes=recv_splits,
                           input_split_sizes=send_splits, group=group)
    return out.to(ids.device)


def build_communication_pattern(
    global_edge_list: torch.Tensor,
    partitioning: torch.Tensor,
    rank: int,
    world_size: int,
    neighbor_partitioning: Optional[torch.Tensor] = None,
    group: Optional[dist.ProcessGroup] = None,
) -> CommunicationPattern:
    """Build the halo pattern of ``rank`` (collective over ``group``).

    ``global_edge_list[E, 2]`` holds (central, neighbor) pairs; ``partitioning`` places
    central vertices, ``neighbor_partitioning`` (default: same) places neighbor vertices.
    Only the edges of local central vertices are used, so callers may pass just those.
    """
    dev = global_edge_list.device
    nbr_part = partitioning if neighbor_partitioning is None else neighbor_partitioning
    local_c = compute_local_vertices(partitioning, rank)
    local_n = local_c if neighbor_partitioning is None else compute_local_vertices(nbr_part, rank)
    L_c, L_n = local_c.numel(), local_n.numel()

    mine = global_edge_list[partitioning[global_edge_list[:, 0]] == rank]
    nbr = mine[:, 1]
    nbr_owner = nbr_part[nbr]
    remote = nbr_owner != rank
    V_n = nbr_part.numel()
    # halo in receive order: (owner, gid) ascending
    key = torch.unique(nbr_owner[remote] * V_n + nbr[remote])
    halo_owner = torch.div(key, V_n, rounding_mode="floor")
    halo = key - halo_owner * V_n
    H = halo.numel()

    g2l_c = _inverse_map(local_c, partitioning.numel())
    g2l_n = _inverse_map(local_n, V_n)
    g2l_n[halo] = torch.arange(L_n, L_n + H, device=dev)
    local_edge_list = torch.stack([g2l_c[mine[:, 0]], g2l_n[nbr]], dim=1)

    req_counts = torch.bincount(halo_owner, minlength=world_size) if H else \
        torch.zeros(world_size, dtype=torch.long, device=dev)
    if world_size > 1 and dist.is_initialized():
        send_counts = _alltoall_counts(req_counts, group)
        wanted = _alltoallv_ids(halo, req_counts.tolist(), send_counts.tolist(), group)
    else:
        send_counts = torch.zeros_like(req_counts)
        wanted = halo[:0]
    send_local_idx = g2l_n[wanted] if wanted.numel() else torch.zeros(0, dtype=torch.long, device=dev)
    if send_local_idx.numel() and bool((send_local_idx < 0).any()) or \
            (send_local_idx.numel() and bool((send_local_idx >= L_n).any())):
        raise RuntimeError("halo request for a vertex this rank does not own")
    send_offset = torch.zeros(world_size + 1, dtype=torch.long, device=dev)
    send_offset[1:] = torch.cumsum(send_counts.to(dev), 0)
    comm_map = compute_comm_map(send_offset, world_size, group)
    recv_offset, _ = compute_recv_offsets(comm_map, rank)
    return CommunicationPattern(
        rank=rank,
        world_size=world_size,
        num_local_vertices=L_c,
        num_halo_vertices=H,
        local_edge_list=local_edge_list,
        send_local_idx=send_local_idx,
        send_offset=send_offset,
        recv_offset=recv_offset,
        comm_map=comm_map,
        put_forward_remote_offset=comm_map[:rank, :].sum(0),
        put_backward_remote_offset=comm_map[:, :rank].sum(1),
        halo_vertices=halo,
        local_vertices=local_c,
        num_local_neighbor_vertices=L_n,
    )


# --------------------------------------------------------------------------------------
# Offline builder: every rank's pattern in one process (no process group)
# --------------------------------------------------------------------------------------
def build_all_patterns_offline(
    global_edge_list: torch.Tensor,
    partitioning: torch.Tensor,
    world_size: int,
    neighbor_partitioning: Optional[torch.Tensor] = None,
) -> List[CommunicationPattern]:
    """The patterns :func:`build_communication_pattern` would produce on each of
    ``world_size`` ranks, computed in ONE process with the two collectives (request-count
    all-to-all, id all-to-all-v) and the comm-map all-gather carried out in memory.

    This is the plan-cache generator of the reference (experiments/OGB/GenerateCache.py,
    OGB-LSC/CacheGenerator.py:119-170 with its dummy communicator) as a library call:
    plans for a W-rank job can be built and saved on one host and loaded by each rank
    (:func:`save_patterns` / :func:`load_pattern`)."""
    dev = global_edge_list.device
    W = int(world_size)
    nbr_part = partitioning if neighbor_partitioning is None else neighbor_partitioning
    V_c, V_n = partitioning.numel(), nbr_part.numel()
    per = []
    for r in range(W):
        local_c = compute_local_vertices(partitioning, r)
        local_n = local_c if neighbor_partitioning is None else compute_local_vertices(nbr_part, r)
        mine = global_edge_list[partitioning[global_edge_list[:, 0]] == r]
        nbr = mine[:, 1]
        owner = nbr_part[nbr]
        remote = owner != r
        key = torch.unique(owner[remote] * V_n + nbr[remote])
        h_owner = torch.div(key, V_n, rounding_mode="floor")
        halo = key - h_owner * V_n
        req = torch.bincount(h_owner, minlength=W) if halo.numel() else \
            torch.zeros(W, dtype=torch.long, device=dev)
        g2l_c = _inverse_map(local_c, V_c)
        g2l_n = _inverse_map(local_n, V_n)
        g2l_n[halo] = torch.arange(local_n.numel(), local_n.numel() + halo.numel(), device=dev)
        per.append(dict(local_c=local_c, local_n=local_n, mine=mine, halo=halo,
                        h_owner=h_owner, req=req, g2l_c=g2l_c, g2l_n=g2l_n))
    # comm_map[q, p] = rows q sends to p = ids p requests from q
    comm_map = torch.stack([per[p]["req"] for p in range(W)], dim=1).long()
    out = []
    for q in range(W):
        P = per[q]
        # what q sends, peer order: the ids each peer p requested from q (p's receive order)
        wanted = [per[p]["halo"][per[p]["h_owner"] == q] for p in range(W)]
        wanted = torch.cat(wanted) if wanted else P["halo"][:0]
        send_local_idx = P["g2l_n"][wanted] if wanted.numel() else \
            torch.zeros(0, dtype=torch.long, device=dev)
        if send_local_idx.numel() and bool(((send_local_idx < 0) |
                                            (send_local_idx >= P["local_n"].numel())).any()):
            raise RuntimeError("halo request for a vertex the sender does not own")
        send_offset = torch.zeros(W + 1, dtype=torch.long, device=dev)
        send_offset[1:] = torch.cumsum(comm_map[q].to(dev), 0)
        recv_offset, _ = compute_recv_offsets(comm_map, q)
        mine = P["mine"]
        out.append(CommunicationPattern(
            rank=q, world_size=W,
            num_local_vertices=P["local_c"].numel(),
            num_halo_vertices=P["halo"].numel(),
            local_edge_list=torch.stack([P["g2l_c"][mine[:, 0]], P["g2l_n"][mine[:, 1]]], 1),
            send_local_idx=send_local_idx,
            send_offset=send_offset,
            recv_offset=recv_offset,
            comm_map=comm_map.clone(),
            put_forward_remote_offset=comm_map[:q, :].sum(0),
            put_backward_remote_offset=comm_map[:, :q].sum(1),
            halo_vertices=P["halo"],
            local_vertices=P["local_c"],
            num_local_neighbor_vertices=P["local_n"].numel(),
        ))
    return out


_PATTERN_TENSORS = ("local_edge_list", "send_local_idx", "send_offset", "recv_offset",
                    "comm_map", "put_forward_remote_offset", "put_backward_remote_offset",
                    "halo_vertices", "local_vertices")
_PATTERN_INTS = ("rank", "world_size", "num_local_vertices", "num_halo_vertices",
                 "num_local_neighbor_vertices")


def pattern_to_dict(cp: CommunicationPattern) -> dict:
    """Plain tensors + ints (loadable with ``torch.load(weights_only=True)``, no pickled
    classes: SURVEY.md §5.4)."""
    d = {k: getattr(cp, k) for k in _PATTERN_TENSORS if getattr(cp, k) is not None}
    d.update({k: int(getattr(cp, k)) for k in _PATTERN_INTS if getattr(cp, k) is not None})
    return d


def pattern_from_dict(d: dict) -> CommunicationPattern:
    return CommunicationPattern(**{k: d[k] for k in _PATTERN_TENSORS + _PATTERN_INTS if k in d})


def save_patterns(patterns: List[CommunicationPattern], directory: str, name: str) -> List[str]:
    """``{directory}/{name}_rank_{r}_of_{W}_comm_pattern.pt`` per rank (the reference's
    per-rank plan file naming, distributed_graph_dataset.py:399-410)."""
    import os

    os.makedirs(directory, exist_ok=True)
    paths = []
    for cp in patterns:
        p = os.path.join(directory, f"{name}_rank_{cp.rank}_of_{cp.world_size}_comm_pattern.pt")
        torch.save(pattern_to_dict(cp), p)
        paths.append(p)
    return paths


def load_pattern(directory: str, name: str, rank: int, world_size: int,
                 map_location="cpu") -> CommunicationPattern:
    import os

    p = os.path.join(directory, f"{name}_rank_{rank}_of_{world_size}_comm_pattern.pt")
    return pattern_from_dict(torch.load(p, map_location=map_location, weights_only=True))
