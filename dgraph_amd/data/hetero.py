"""Heterogeneous (MAG-like) distributed graphs for the OGB-LSC RGAT experiment.

Counterparts of ``DistributedHeteroGraphDataset`` / ``SyntheticHeterogeneousDataset`` /
``DGraph_MAG240M_Dataset`` (experiments/OGB-LSC/lsc_datasets/*.py). Node types are
0 = paper, 1 = author, 2 = institution, each split into contiguous per-rank blocks
(``get_vertex_offsets``). The five relations are the reference's
``edge_type = [(0,0), (0,1), (1,0), (1,2), (2,1)]`` ((source type, destination type)).

Each relation becomes a :class:`RelationGraph`: a bipartite halo pattern (destination
vertices local, source vertices local or halo, built by the request-based
:func:`build_communication_pattern` with ``neighbor_partitioning`` — the reference's
bipartite builder was stale, D5) plus the destination-sorted CSR the attention kernels
run on. Plans are cached on disk keyed by an md5 of the configuration (the reference's
``synthetic_dataset_{hash}_rank_{r}_of_{W}_comm_plans.pt``), stored as plain tensors.
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from ..ops.csr import CSR, IndexMap
from ..plan.pattern import CommunicationPattern, build_communication_pattern

EDGE_TYPES: List[Tuple[int, int]] = [(0, 0), (0, 1), (1, 0), (1, 2), (2, 1)]
NODE_TYPES = ("paper", "author", "institution")


def get_vertex_offsets(num_vertices: int, world_size: int) -> torch.Tensor:
    """Contiguous block offsets ``[W + 1]`` (first ``V % W`` ranks get one extra)."""
    base, extra = divmod(int(num_vertices), int(world_size))
    sizes = torch.full((world_size,), base, dtype=torch.long)
    sizes[:extra] += 1
    off = torch.zeros(world_size + 1, dtype=torch.long)
    off[1:] = torch.cumsum(sizes, 0)
    return off


def placement_from_offsets(offsets: torch.Tensor) -> torch.Tensor:
    sizes = offsets[1:] - offsets[:-1]
    return torch.repeat_interleave(torch.arange(sizes.numel()), sizes)


@dataclass
class RelationGraph:
    """One relation (src type -> dst type) seen from one rank."""

    src_type: int
    dst_type: int
    pattern: CommunicationPattern
    csr: CSR                      # rows: local dst vertices; cols: [local src | halo]
    num_local_dst: int
    num_local_src: int
    _cache: dict = field(default_factory=dict, repr=False)

    @property
    def num_halo(self) -> int:
        return int(self.pattern.num_halo_vertices)

    def row_map(self) -> IndexMap:
        """Edge slot -> destination row (CSR slot order)."""
        m = self._cache.get("row_map")
        if m is None:
            m = IndexMap(self.csr.row_ids(), self.num_local_dst)
            self._cache["row_map"] = m
        return m

    def col_map(self) -> IndexMap:
        """Edge slot -> source row of ``[local src | halo]`` (CSR slot order)."""
        m = self._cache.get("col_map")
        if m is None:
            m = IndexMap(self.csr.col.long(), self.num_local_src + self.num_halo)
            self._cache["col_map"] = m
        return m

    def to(self, device) -> "RelationGraph":
        self.pattern = self.pattern.to(device)
        self.csr = self.csr.to(device)
        self._cache.clear()
        return self

    def state_dict(self) -> dict:
        p = self.pattern
        return {"src_type": self.src_type, "dst_type": self.dst_type,
                "num_local_dst": self.num_local_dst, "num_local_src": self.num_local_src,
                "rowptr": self.csr.rowptr, "col": self.csr.col,
                "num_cols": self.csr.num_cols, "p_rank": p.rank, "p_world": p.world_size,
                "p_L": p.num_local_vertices, "p_H": p.num_halo_vertices,
                "local_edge_list": p.local_edge_list, "send_local_idx": p.send_local_idx,
                "send_offset": p.send_offset, "recv_offset": p.recv_offset,
                "comm_map": p.comm_map, "fwd": p.put_forward_remote_offset,
                "bwd": p.put_backward_remote_offset, "halo_vertices": p.halo_vertices,
                "local_vertices": p.local_vertices, "p_Ln": p.num_local_neighbor_vertices}

    @staticmethod
    def from_state_dict(d: dict) -> "RelationGraph":
        p = CommunicationPattern(
            rank=d["p_rank"], world_size=d["p_world"], num_local_vertices=d["p_L"],
            num_halo_vertices=d["p_H"], local_edge_list=d["local_edge_list"],
            send_local_idx=d["send_local_idx"], send_offset=d["send_offset"],
            recv_offset=d["recv_offset"], comm_map=d["comm_map"],
            put_forward_remote_offset=d["fwd"], put_backward_remote_offset=d["bwd"],
            halo_vertices=d["halo_vertices"], local_vertices=d["local_vertices"],
            num_local_neighbor_vertices=d["p_Ln"])
        csr = CSR(d["rowptr"], d["col"], d["num_cols"])
        return RelationGraph(d["src_type"], d["dst_type"], p, csr, d["num_local_dst"],
                             d["num_local_src"])


def build_relation_graph(edges: torch.Tensor, src_type: int, dst_type: int,
                         offsets: Dict[int, torch.Tensor], rank: int, world_size: int,
                         group=None) -> RelationGraph:
    """``edges[2, E]`` = (global src id, global dst id) of one relation (collective)."""
    src_part = placement_from_offsets(offsets[src_type])
    dst_part = placement_from_offsets(offsets[dst_type])
    el = torch.stack([edges[1], edges[0]], dim=1).long()  # (central = dst, neighbour = src)
    cp = build_communication_pattern(el, dst_part, rank, world_size,
                                     neighbor_partitioning=src_part, group=group)
    Ld = int(offsets[dst_type][rank + 1] - offsets[dst_type][rank])
    Ls = int(offsets[src_type][rank + 1] - offsets[src_type][rank])
    lel = cp.local_edge_list
    csr = CSR.from_coo(lel[:, 0], lel[:, 1], Ld, Ls + int(cp.num_halo_vertices),
                       keep_perm=False)
    return RelationGraph(src_type, dst_type, cp, csr, Ld, Ls)


# ----------------------------------------------------------------------------- synthetic MAG
def _generator(seed: int) -> torch.Generator:
    return torch.Generator().manual_seed(int(seed))


def paper_2_paper_edges(num_papers: int, seed: int = 0) -> torch.Tensor:
    """~11 citations per paper, de-duplicated and symmetrised (synthetic_dataset.py:38-48)."""
    g = _generator(seed)
    e = torch.randint(0, num_papers, (2, num_papers * 11), generator=g)
    e = torch.unique(e, dim=1)
    return torch.unique(torch.cat([e, e.flip(0)], dim=1), dim=1)


def author_2_paper_edges(num_authors: int, num_papers: int, seed: int = 1) -> torch.Tensor:
    """~3.5 papers per author (synthetic_dataset.py:51-62)."""
    g = _generator(seed)
    n = int(num_authors * 3.5)
    e = torch.stack([torch.randint(0, num_authors, (n,), generator=g),
                     torch.randint(0, num_papers, (n,), generator=g)])
    return torch.unique(e, dim=1)


def author_2_institution_edges(num_authors: int, num_institutions: int,
                               seed: int = 2) -> torch.Tensor:
    """~0.35 institutions per author (synthetic_dataset.py:65-76)."""
    g = _generator(seed)
    n = max(1, int(num_authors * 0.35))
    e = torch.stack([torch.randint(0, num_authors, (n,), generator=g),
                     torch.randint(0, num_institutions, (n,), generator=g)])
    return torch.unique(e, dim=1)


@dataclass
class SyntheticHeteroConfig:
    """SyntheticDatasetConfig (experiments/OGB-LSC/config.py:38-45)."""

    num_papers: int = 2048
    num_authors: int = 8192
    num_institutions: int = 256
    num_features: int = 768
    num_classes: int = 153
    seed: int = 0


def config_hash(values) -> str:
    return hashlib.md5(str(tuple(values)).encode("utf-8")).hexdigest()


class DistributedHeteroGraphDataset:
    """Per-rank view of a 3-type heterogeneous graph with one :class:`RelationGraph`
    per edge type."""

    num_node_types = 3

    def __init__(self, rank: int, world_size: int, num_features: int, num_classes: int,
                 features: List[torch.Tensor], offsets: Dict[int, torch.Tensor],
                 labels: torch.Tensor, split: Dict[str, torch.Tensor],
                 relations: List[RelationGraph]):
        self.rank, self.world_size = rank, world_size
        self._num_features, self._num_classes = num_features, num_classes
        self._num_relations = len(relations)
        self.features = features
        self.offsets = offsets
        self.y = labels                 # global paper labels
        self.split = split              # global paper ids per split
        self.relations = relations
        self.edge_types = [(r.src_type, r.dst_type) for r in relations]

    @property
    def num_features(self) -> int:
        return self._num_features

    @property
    def num_classes(self) -> int:
        return self._num_classes

    @property
    def num_relations(self) -> int:
        return self._num_relations

    def __len__(self) -> int:
        return 1

    def __getitem__(self, idx):
        return self.features, self.edge_types, self.relations

    def to(self, device) -> "DistributedHeteroGraphDataset":
        self.features = [f.to(device) for f in self.features]
        self.relations = [r.to(device) for r in self.relations]
        self.y = self.y.to(device)
        self.split = {k: v.to(device) for k, v in self.split.items()}
        return self

    def get_mask(self, mask_type: str) -> torch.Tensor:
        """Local row indices of this rank's papers in the ``train``/``val``/``test`` split."""
        ids = self.split[mask_type].long()
        lo, hi = int(self.offsets[0][self.rank]), int(self.offsets[0][self.rank + 1])
        return ids[(ids >= lo) & (ids < hi)] - lo

    def get_target(self, mask_type: str) -> torch.Tensor:
        ids = self.split[mask_type].long()
        lo, hi = int(self.offsets[0][self.rank]), int(self.offsets[0][self.rank + 1])
        return self.y[ids[(ids >= lo) & (ids < hi)]]


class SyntheticHeterogeneousDataset(DistributedHeteroGraphDataset):
    """MAG240M-like synthetic graph (synthetic_dataset.py:79-199). Every rank generates the
    same global edge lists from fixed seeds and keeps its own feature rows; features are
    drawn per global vertex (seeded by type), so results do not depend on W."""

    def __init__(self, config: SyntheticHeteroConfig, comm, cache_dir: Optional[str] = None):
        rank, W = comm.get_rank(), comm.get_world_size()
        c = config
        counts = [c.num_papers, c.num_authors, c.num_institutions]
        offsets = {t: get_vertex_offsets(n, W) for t, n in enumerate(counts)}
        g = _generator(c.seed + 17)
        perm = torch.randperm(c.num_papers, generator=g)
        n_tr, n_va = int(0.7 * c.num_papers), int(0.85 * c.num_papers)
        split = {"train": perm[:n_tr], "val": perm[n_tr:n_va], "test": perm[n_va:]}
        labels = torch.randint(0, c.num_classes, (c.num_papers,), generator=g)
        feats = []
        for t, n in enumerate(counts):
            lo, hi = int(offsets[t][rank]), int(offsets[t][rank + 1])
            gt = _generator(c.seed * 1000 + 31 * t + 5)
            full = torch.randn(n, c.num_features, generator=gt)  # small synthetic scales
            feats.append(full[lo:hi].contiguous())
        relations = self._relations(c, comm, offsets, rank, W, cache_dir)
        super().__init__(rank, W, c.num_features, c.num_classes, feats, offsets, labels, split,
                         relations)

    @staticmethod
    def _relations(c, comm, offsets, rank, W, cache_dir) -> List[RelationGraph]:
        path = None
        if cache_dir is not None:
            h = config_hash([c.num_papers, c.num_authors, c.num_institutions, c.num_features,
                             c.num_classes, c.seed])
            path = os.path.join(cache_dir,
                                f"synthetic_dataset_{h}_rank_{rank}_of_{W}_comm_plans.pt")
            if os.path.exists(path):
                d = torch.load(path, weights_only=True)
                return [RelationGraph.from_state_dict(x) for x in d["relations"]]
        p2p = paper_2_paper_edges(c.num_papers, c.seed)
        a2p = author_2_paper_edges(c.num_authors, c.num_papers, c.seed + 1)
        a2i = author_2_institution_edges(c.num_authors, c.num_institutions, c.seed + 2)
        rel_edges = {(0, 0): p2p, (0, 1): a2p.flip(0), (1, 0): a2p, (1, 2): a2i,
                     (2, 1): a2i.flip(0)}
        group = getattr(comm, "group", None)
        rels = [build_relation_graph(rel_edges[et], et[0], et[1], offsets, rank, W, group)
                for et in EDGE_TYPES]
        if path is not None:
            os.makedirs(cache_dir, exist_ok=True)
            torch.save({"relations": [r.state_dict() for r in rels]}, path)
        return rels


def derive_features_by_mean(src_feats_global: torch.Tensor, edges: torch.Tensor,
                            num_dst: int) -> torch.Tensor:
    """Features of a featureless type as the mean of its neighbours' features
    (MAG240M_dataset.py:65-102: author = mean of written papers, institution = mean of
    affiliated authors). ``edges[2, E]`` = (src, dst)."""
    from ..ops.aggregate import aggregate

    csr = CSR.from_coo(edges[1].long(), edges[0].long(), num_dst, src_feats_global.shape[0])
    return aggregate(src_feats_global, csr, reduce="mean")


def __getattr__(name):
    # The real-MAG240M dataset reads the on-disk layout directly (no ``ogb``):
    # data/mag240m.py (imported lazily: it builds on this module).
    if name == "DGraph_MAG240M_Dataset":
        from .mag240m import DGraph_MAG240M_Dataset
        return DGraph_MAG240M_Dataset
    raise AttributeError(name)
