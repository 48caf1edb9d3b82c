"""``DistributedOGBWrapper`` (DGraph/data/ogbn_datasets.py:25-148 API).

Loads an OGB node-property dataset on rank 0 first (barriers around it, avoiding the
download/processing race the reference describes), builds a contiguous-ownership
:class:`DistributedGraph` and caches it at ``{dir}/{dname}_graph_data_{W}.pt`` (the
reference's file name; stored as plain tensors, loaded with ``weights_only=True``).

The ``ogb`` package is not installed in this environment and there is no network: when it
is missing, the wrapper builds a *synthetic* graph of the dataset's published shape
(:mod:`dgraph_amd.data.synthetic`) and says so (``self.synthetic = True``). Pass
``allow_synthetic=False`` to require the real dataset.
"""
from __future__ import annotations

import os
import warnings
from typing import Optional

import torch

from .graph import DistributedGraph, get_round_robin_node_rank_map
from .preprocess import process_homogenous_data

SUPPORTED_DATASETS = ["ogbn-arxiv", "ogbn-proteins", "ogbn-papers100M", "ogbn-products"]
num_classes = {"ogbn-arxiv": 40, "ogbn-proteins": 112, "ogbn-papers100M": 172,
               "ogbn-products": 47}


def _load_ogb(dname: str, root: str):
    from ogb.nodeproppred import NodePropPredDataset  # type: ignore

    ds = NodePropPredDataset(name=dname, root=root)
    graph, labels = ds[0]
    return graph, labels, ds.get_idx_split()


def _synthetic_ogb(dname: str, scale: float = 1.0, seed: int = 0):
    """Global synthetic graph in OGB dict form (small scales only: holds the global
    edge list in host memory, like the reference's loaders did)."""
    from .synthetic import SHAPES, build_local_csr, node_data

    shape = SHAPES[dname] if scale == 1.0 else SHAPES[dname].scaled(scale)
    csr, L, off = build_local_csr(shape, 0, 1, "cpu", seed=seed)
    rows = csr.row_ids()
    edge_index = torch.stack([rows, csr.col.long()])
    x, y, train = node_data(shape, 0, off, "cpu", seed=seed, dtype=torch.float32)
    g = torch.Generator().manual_seed(seed)
    perm = torch.randperm(L, generator=g)
    n_tr = int(train.sum())
    n_va = max(1, (L - n_tr) // 2)
    split = {"train": perm[:n_tr].numpy(), "valid": perm[n_tr:n_tr + n_va].numpy(),
             "test": perm[n_tr + n_va:].numpy()}
    graph = {"node_feat": x.numpy(), "edge_index": edge_index.numpy(), "num_nodes": L,
             "edge_feat": None}
    return graph, y.numpy(), split


class DistributedOGBWrapper(torch.utils.data.Dataset):
    def __init__(self, dname: str, comm_object, dir_name: Optional[str] = None,
                 node_rank_placement: Optional[torch.Tensor] = None,
                 force_reprocess: bool = False, allow_synthetic: bool = True,
                 synthetic_scale: float = 1.0, *args, **kwargs) -> None:
        super().__init__()
        if dname not in SUPPORTED_DATASETS:
            raise AssertionError(f"Dataset {dname} not supported. Supported: {SUPPORTED_DATASETS}")
        self.dname = dname
        self.num_classes = num_classes[dname]
        self.comm_object = comm_object
        self._rank = comm_object.get_rank()
        self._world_size = comm_object.get_world_size()
        dir_name = dir_name if dir_name is not None else os.path.join(os.getcwd(), "data")
        os.makedirs(dir_name, exist_ok=True)
        cached = os.path.join(dir_name, f"{dname}_graph_data_{self._world_size}.pt")
        self.synthetic = False
        if os.path.exists(cached) and not force_reprocess:
            self.graph_obj = DistributedGraph.load(cached)
            return
        graph = labels = split = None
        comm_object.barrier()
        for turn in (0, 1):  # rank 0 first, then everyone else (download race)
            if (self._rank == 0) == (turn == 0):
                try:
                    graph, labels, split = _load_ogb(dname, dir_name)
                except ImportError:
                    if not allow_synthetic:
                        raise
                    if self._rank == 0:
                        warnings.warn(f"ogb is not installed: using a synthetic {dname}-shaped "
                                      f"graph (scale {synthetic_scale})")
                    graph, labels, split = _synthetic_ogb(dname, synthetic_scale)
                    self.synthetic = True
            comm_object.barrier()
        if node_rank_placement is None:
            node_rank_placement = get_round_robin_node_rank_map(int(graph["num_nodes"]),
                                                                self._world_size)
        self.split_idx = split
        self.graph_obj = process_homogenous_data(graph, labels, self._rank, self._world_size,
                                                 split, node_rank_placement, *args, **kwargs)
        if self._rank == 0:
            self.graph_obj.save(cached)
        comm_object.barrier()

    def __len__(self) -> int:
        return 1

    def __getitem__(self, idx: int):
        rank = self.comm_object.get_rank()
        x = self.graph_obj.get_local_node_features(rank=rank)
        y = self.graph_obj.get_local_labels(rank=rank)
        if getattr(self.comm_object, "backend", "nccl") in ("nccl", "gloo"):
            # two-sided G1 form: global edge list + (placement, owner) mappings
            return (x, self.graph_obj.get_global_edge_indices(),
                    self.graph_obj.get_global_rank_mappings(), y)
        return (x, self.graph_obj.get_local_edge_indices(rank=rank),
                self.graph_obj.get_local_rank_mappings(rank=rank), y)
