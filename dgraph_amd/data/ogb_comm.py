"""``DGraphOGBDataset`` — OGB node-property data with a halo communication pattern
(experiments/OGB/ogb_comm_dataset.py:14-145 API).

Rank 0 loads first (barriers around it), every rank then builds its
:class:`~dgraph_amd.plan.pattern.CommunicationPattern` for the given vertex placement
(round-robin by default) and keeps its local features, labels and split masks. Local
vertices are the placement's vertices of this rank in increasing global id (the
reference's order). When ``ogb`` is not installed, a synthetic graph of the dataset's
published shape is used (``self.synthetic``; see :mod:`dgraph_amd.data.ogbn`).
"""
from __future__ import annotations

import warnings
from typing import Dict, Optional

import torch

from ..plan.pattern import CommunicationPattern, build_communication_pattern
from .graph import get_round_robin_node_rank_map
from .ogbn import SUPPORTED_DATASETS, _load_ogb, _synthetic_ogb, num_classes


def build_local_split_masks(node_rank_placement: torch.Tensor, split_idx: dict,
                            rank: int) -> Dict[str, torch.Tensor]:
    """Global split index lists -> boolean masks over this rank's local vertices."""
    V = node_rank_placement.shape[0]
    local_ids = torch.nonzero(node_rank_placement == rank).reshape(-1)
    masks = {}
    for name, ids in split_idx.items():
        g = torch.zeros(V, dtype=torch.bool)
        g[torch.as_tensor(ids).long()] = True
        masks[name] = g[local_ids]
    return masks


def generate_communication_pattern(edge_index: torch.Tensor, node_rank_placement: torch.Tensor,
                                   rank: int, world_size: int, group=None
                                   ) -> CommunicationPattern:
    return build_communication_pattern(edge_index, node_rank_placement, rank, world_size,
                                       group=group)


class DGraphOGBDataset(torch.utils.data.Dataset):
    def __init__(self, dname: str, comm, node_rank_placement: Optional[torch.Tensor] = None,
                 root_dir: Optional[str] = None, allow_synthetic: bool = True,
                 synthetic_scale: float = 1.0, *args, **kwargs) -> None:
        super().__init__()
        if dname not in SUPPORTED_DATASETS:
            raise ValueError(f"unsupported dataset {dname}; choose from {SUPPORTED_DATASETS}")
        self.comm_object = comm
        self.rank = comm.get_rank()
        self.world_size = comm.get_world_size()
        self.num_classes = num_classes[dname]
        self.synthetic = False
        root = root_dir or "dataset"
        graph = labels = split = None
        comm.barrier()
        for turn in (0, 1):
            if (self.rank == 0) == (turn == 0):
                try:
                    graph, labels, split = _load_ogb(dname, root)
                except ImportError:
                    if not allow_synthetic:
                        raise
                    if self.rank == 0:
                        warnings.warn(f"ogb is not installed: synthetic {dname}-shaped graph "
                                      f"(scale {synthetic_scale})")
                    graph, labels, split = _synthetic_ogb(dname, synthetic_scale)
                    self.synthetic = True
            comm.barrier()
        V = int(graph["num_nodes"])
        x = torch.as_tensor(graph["node_feat"]).float()
        edge_index = torch.as_tensor(graph["edge_index"]).long().t().contiguous()
        y = torch.as_tensor(labels).long().reshape(V, -1)
        if y.shape[1] == 1:
            y = y[:, 0]
        if node_rank_placement is None:
            node_rank_placement = get_round_robin_node_rank_map(V, self.world_size)
        node_rank_placement = node_rank_placement.long()
        self.node_rank_placement = node_rank_placement
        self.comm_pattern = generate_communication_pattern(
            edge_index, node_rank_placement, self.rank, self.world_size,
            group=getattr(comm, "group", None))
        local = node_rank_placement == self.rank
        self.local_node_features = x[local]
        self.local_labels = y[local]
        masks = build_local_split_masks(node_rank_placement,
                                        {k: torch.as_tensor(v) for k, v in split.items()},
                                        self.rank)
        self.train_mask = masks["train"]
        self.val_mask = masks["valid"]
        self.test_mask = masks["test"]
        self.num_global_edges = int(edge_index.shape[0])

    def get_masks(self) -> Dict[str, torch.Tensor]:
        return {"train_mask": self.train_mask, "val_mask": self.val_mask,
                "test_mask": self.test_mask}

    def __len__(self) -> int:
        return 1

    def __getitem__(self, index):
        return self.local_node_features, self.local_labels, self.comm_pattern
