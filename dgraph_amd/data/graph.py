"""``DistributedGraph``: a whole graph plus its vertex/edge placement across ranks.

Same constructor and accessors as the reference container (DGraph/data/graph.py:24-267).
Additions: ``to(device)``, ``save``/``load`` with plain-tensor payloads (safe
``weights_only`` loading instead of pickled classes), ``local_csr(rank)`` and
``communication_pattern(rank)`` shortcuts into the library's plan builders.
"""
from __future__ import annotations

from typing import Optional

import torch


class DistributedGraph:
    def __init__(
        self,
        node_features: torch.Tensor,
        edge_index: torch.Tensor,
        labels: torch.Tensor,
        node_loc: torch.Tensor,
        edge_loc: torch.Tensor,
        edge_dest_rank_mapping: torch.Tensor,
        num_nodes: int,
        num_edges: int,
        world_size: int,
        edge_features: Optional[torch.Tensor] = None,
        train_mask: Optional[torch.Tensor] = None,
        val_mask: Optional[torch.Tensor] = None,
        test_mask: Optional[torch.Tensor] = None,
        graph_labels: Optional[torch.Tensor] = None,
    ):
        if node_features.dim() != 2:
            raise AssertionError("Invalid node features shape. Expect 2D tensor")
        if edge_index.dim() != 2:
            raise AssertionError("Invalid edge index shape. Expect 2D tensor")
        if node_loc.dim() != 1 or edge_loc.dim() != 1:
            raise AssertionError("node_loc / edge_loc must be 1D")
        if node_features.shape[0] != num_nodes or node_loc.shape[0] != num_nodes:
            raise AssertionError(f"expected {num_nodes} nodes, got {node_features.shape}")
        if edge_index.shape[1] != num_edges or edge_loc.shape[0] != num_edges:
            raise AssertionError(f"expected {num_edges} edges, got {edge_index.shape}")
        self.num_nodes = int(num_nodes)
        self.num_edges = int(num_edges)
        self.node_features = node_features
        self.edge_index = edge_index
        self.edge_features = edge_features
        self.labels = labels
        self.train_mask = train_mask
        self.val_mask = val_mask
        self.test_mask = test_mask
        self.graph_labels = graph_labels
        self.world_size = int(world_size)
        self.node_loc = node_loc
        self.edge_loc = edge_loc
        self.edge_dest_rank_mapping = edge_dest_rank_mapping
        self._nodes_per_rank = torch.bincount(node_loc, minlength=world_size)
        self._edges_per_rank = torch.bincount(edge_loc, minlength=world_size)
        self.max_node_per_rank = int(self._nodes_per_rank.max()) if num_nodes else 0
        self.max_edge_per_rank = int(self._edges_per_rank.max()) if num_edges else 0
        self.rank_mappings = torch.stack([edge_loc, edge_dest_rank_mapping], dim=0)

    # -------------------------------------------------------------- accessors
    def get_nodes_per_rank(self) -> torch.Tensor:
        return self._nodes_per_rank

    def get_edges_per_rank(self) -> torch.Tensor:
        return self._edges_per_rank

    def get_max_node_per_rank(self) -> int:
        return self.max_node_per_rank

    def get_max_edge_per_rank(self) -> int:
        return self.max_edge_per_rank

    def get_local_node_features(self, rank) -> torch.Tensor:
        return self.node_features[self.node_loc == rank]

    def get_global_node_features(self) -> torch.Tensor:
        return self.node_features

    def get_local_edge_indices(self, rank) -> torch.Tensor:
        return self.edge_index[:, self.edge_loc == rank]

    def get_global_edge_indices(self) -> torch.Tensor:
        return self.edge_index

    def get_global_rank_mappings(self) -> torch.Tensor:
        return self.rank_mappings

    def get_local_rank_mappings(self, rank) -> torch.Tensor:
        return self.rank_mappings[:, self.edge_loc == rank]

    def get_local_labels(self, rank) -> torch.Tensor:
        return self.labels[self.node_loc == rank]

    def get_global_labels(self) -> torch.Tensor:
        return self.labels

    def local_node_range(self, rank) -> tuple:
        """[start, end) of ``rank``'s vertices (valid after contiguous renumbering, I1)."""
        start = int(self._nodes_per_rank[:rank].sum())
        return start, start + int(self._nodes_per_rank[rank])

    def get_local_mask(self, mask: str, rank) -> torch.Tensor:
        """Local indices of the ``train``/``val``/``test`` vertices owned by ``rank``."""
        m = {"train": self.train_mask, "val": self.val_mask, "test": self.test_mask}.get(mask, ...)
        if m is ...:
            raise ValueError(f"Invalid mask {mask}")
        if m is None:
            raise AssertionError(f"{mask} mask not found")
        start, end = self.local_node_range(rank)
        m = m.long()
        sel = (m >= start) & (m < end)
        return m[sel] - start

    def _get_index_to_rank_mapping(self, indices):
        return self.node_loc[indices.long()]

    def get_sender_receiver_ranks(self):
        return self.edge_loc, self.edge_dest_rank_mapping

    # -------------------------------------------------------------- extensions
    def to(self, device) -> "DistributedGraph":
        for k, v in list(self.__dict__.items()):
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device))
        return self

    def local_csr(self, rank: int, reduce_at: str = "src"):
        """CSR of this rank's edges: rows = the owned central vertex (local index),
        columns = global ids of the other endpoint."""
        from ..ops.csr import CSR

        start, end = self.local_node_range(rank)
        ei = self.get_local_edge_indices(rank)
        central, nbr = (ei[0], ei[1]) if reduce_at == "src" else (ei[1], ei[0])
        return CSR.from_coo(central - start, nbr, end - start, self.num_nodes)

    def communication_pattern(self, rank: int, group=None):
        """Halo pattern for ``rank`` (edges are (source, destination); the source is the
        central vertex, as in the reference's GCN, GCN.py:57-65)."""
        from ..plan.pattern import build_communication_pattern

        return build_communication_pattern(self.edge_index.t().contiguous(), self.node_loc,
                                           rank, self.world_size, group=group)

    def state_dict(self) -> dict:
        return {k: v for k, v in self.__dict__.items()
                if isinstance(v, (torch.Tensor, int)) and not k.startswith("_")}

    def save(self, path) -> None:
        torch.save(self.state_dict(), path)

    @staticmethod
    def load(path, map_location="cpu") -> "DistributedGraph":
        d = torch.load(path, map_location=map_location, weights_only=True)
        return DistributedGraph(
            node_features=d["node_features"], edge_index=d["edge_index"], labels=d["labels"],
            node_loc=d["node_loc"], edge_loc=d["edge_loc"],
            edge_dest_rank_mapping=d["edge_dest_rank_mapping"], num_nodes=d["num_nodes"],
            num_edges=d["num_edges"], world_size=d["world_size"],
            edge_features=d.get("edge_features"), train_mask=d.get("train_mask"),
            val_mask=d.get("val_mask"), test_mask=d.get("test_mask"),
            graph_labels=d.get("graph_labels"))


def get_round_robin_node_rank_map(num_nodes: int, world_size: int) -> torch.Tensor:
    """Vertex ``i`` -> rank ``i mod world_size`` (vectorised; the reference looped)."""
    if num_nodes < 0:
        raise AssertionError("num_nodes must be non-negative")
    if world_size < 1:
        raise AssertionError("world_size must be at least 1")
    return torch.arange(num_nodes, dtype=torch.long) % world_size
