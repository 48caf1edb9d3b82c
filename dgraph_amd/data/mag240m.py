"""MAG240M from its on-disk layout, without the ``ogb`` package.

Counterpart of ``DGraph_MAG240M_Dataset`` (experiments/OGB-LSC/lsc_datasets/
MAG240M_dataset.py:116-320). ``ogb`` is not importable here, so the dataset directory
written by ``ogb.lsc.MAG240MDataset`` is read directly:

    <root>/mag240m_kddcup2021/             (or <root> itself)
        meta.pt                            {'paper': N_p, 'author': N_a, 'institution': N_i}
        split_dict.pt                      {'train', 'valid', 'test-dev', ...: int64 arrays}
        processed/paper/node_feat.npy      float16 [N_p, 768]   (memory-mapped, ~175 GB)
        processed/paper/node_label.npy     float   [N_p]        (NaN = unlabelled)
        processed/paper___cites___paper/edge_index.npy              int64 [2, E]
        processed/author___writes___paper/edge_index.npy            int64 [2, E]
        processed/author___affiliated_with___institution/edge_index.npy

The two ``.pt`` files are read with ``torch.load(weights_only=True)`` (numpy arrays
admitted through ``torch.serialization.safe_globals``; nothing from the file is executed),
every ``.npy`` with ``numpy.load`` (``allow_pickle=False``) memory-mapped, so a rank only
pages in its own feature rows.

Author and institution features do not exist in MAG240M; as in ogb's ``rgnn.py`` (and the
reference's ``generate_feature_data``) they are derived once by rank 0:
``author = mean of written papers``, ``institution = mean of affiliated authors`` (the
reference fed the paper features and the author count into the institution pass; here the
institution pass aggregates the author features it just wrote). The output files are real
``.npy`` files (``numpy.lib.format.open_memmap``), written in 64-column slices through the
library's CSR mean aggregation (on the GPU when one is present).

Per-rank communication plans are cached as ``MAG240M_dataset_rank_{r}_of_{W}_comm_plans.pt``
in the dataset directory (reference :249-260) with the reference's key names
(``paper_2_paper_comm_plan`` ...), holding plain-tensor state dicts of the
:class:`~dgraph_amd.data.hetero.RelationGraph` of each relation.
"""
from __future__ import annotations

import os
import os.path as osp
from typing import Dict, Optional

import numpy as np
import torch

from ..ops.csr import CSR
from .hetero import (EDGE_TYPES, DistributedHeteroGraphDataset, RelationGraph,
                     build_relation_graph, get_vertex_offsets)

NUM_CLASSES = 153
NUM_PAPER_FEATURES = 768
PLAN_KEYS = {(0, 0): "paper_2_paper_comm_plan", (0, 1): "paper_2_author_comm_plan",
             (1, 0): "author_2_paper_comm_plan", (1, 2): "author_2_institution_comm_plan",
             (2, 1): "institution_2_author_comm_plan"}
_REL_DIRS = {"cites": "paper___cites___paper", "writes": "author___writes___paper",
             "affiliated_with": "author___affiliated_with___institution"}


def _safe_load(path: str):
    """``torch.load(weights_only=True)`` that also admits plain numpy arrays."""
    try:
        recon = np._core.multiarray._reconstruct  # numpy >= 2
    except AttributeError:  # pragma: no cover - numpy 1.x
        recon = np.core.multiarray._reconstruct
    allowed = [recon, np.ndarray, np.dtype, type(np.dtype(np.int64)),
               type(np.dtype(np.int32)), type(np.dtype(np.float32))]
    with torch.serialization.safe_globals(allowed):
        return torch.load(path, weights_only=True, map_location="cpu")


class MAG240MFiles:
    """Read-only view of the MAG240M directory layout (no ``ogb``)."""

    def __init__(self, root: str):
        sub = osp.join(root, "mag240m_kddcup2021")
        self.dir = sub if osp.isdir(sub) else root
        meta_path = osp.join(self.dir, "meta.pt")
        if osp.exists(meta_path):
            meta = _safe_load(meta_path)
            self.num_papers = int(meta["paper"])
            self.num_authors = int(meta["author"])
            self.num_institutions = int(meta["institution"])
        else:  # infer from the arrays
            self.num_papers = int(self.paper_label.shape[0])
            self.num_authors = int(self.edge_index("author", "writes", "paper")[0].max()) + 1
            self.num_institutions = int(
                self.edge_index("author", "affiliated_with", "institution")[1].max()) + 1
        self._split = None

    # --- arrays -----------------------------------------------------------------------
    def _npy(self, *parts) -> np.ndarray:
        return np.load(osp.join(self.dir, "processed", *parts), mmap_mode="r")

    @property
    def paper_feat(self) -> np.ndarray:
        return self._npy("paper", "node_feat.npy")

    @property
    def paper_label(self) -> np.ndarray:
        return self._npy("paper", "node_label.npy")

    @property
    def num_classes(self) -> int:
        return NUM_CLASSES

    def edge_index(self, src: str, rel: str, dst: Optional[str] = None) -> np.ndarray:
        """``edge_index("paper", "cites", "paper")`` / ``("author", "writes", "paper")`` /
        ``("author", "institution")`` (the ogb shorthand) / ``("author", "paper")``."""
        if dst is None:  # two-argument shorthand: (src type, dst type)
            rel, dst = {("author", "paper"): "writes", ("author", "institution"):
                        "affiliated_with", ("paper", "paper"): "cites"}[(src, rel)], rel
        return self._npy(_REL_DIRS[rel], "edge_index.npy")

    def get_idx_split(self, name: str) -> np.ndarray:
        if self._split is None:
            self._split = _safe_load(osp.join(self.dir, "split_dict.pt"))
        return np.asarray(self._split[name])


def _mean_into(out: np.ndarray, src: np.ndarray, edges: np.ndarray, num_dst: int,
               device, col_chunk: int = 64) -> None:
    """``out[d] = mean_{(s, d) in edges} src[s]`` column slice by column slice (``edges``
    is (src id, dst id)); rows without neighbours stay zero."""
    from ..ops.aggregate import aggregate

    e = torch.from_numpy(np.array(edges, dtype=np.int64))
    csr = CSR.from_coo(e[1], e[0], num_dst, src.shape[0]).to(device)
    del e
    for c0 in range(0, src.shape[1], col_chunk):
        c1 = min(c0 + col_chunk, src.shape[1])
        x = torch.from_numpy(np.array(src[:, c0:c1], dtype=np.float32)).to(device)
        out[:, c0:c1] = aggregate(x, csr, reduce="mean").cpu().numpy().astype(out.dtype)
        del x
    if hasattr(out, "flush"):
        out.flush()


def generate_feature_data(files: MAG240MFiles, comm=None, device=None) -> Dict[str, str]:
    """Write ``author_feat.npy`` / ``institution_feat.npy`` (float16, 768 columns) next to
    the dataset if missing (rank 0 only; everyone then waits at a barrier)."""
    rank = comm.get_rank() if comm is not None else 0
    dev = device or (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    pa = osp.join(files.dir, "author_feat.npy")
    pi = osp.join(files.dir, "institution_feat.npy")
    if rank == 0:
        pf = files.paper_feat
        if not osp.exists(pa):
            tmp = pa + ".tmp.npy"
            out = np.lib.format.open_memmap(tmp, mode="w+", dtype=np.float16,
                                            shape=(files.num_authors, pf.shape[1]))
            _mean_into(out, pf, files.edge_index("author", "writes", "paper")[::-1],
                       files.num_authors, dev)
            del out
            os.replace(tmp, pa)
        if not osp.exists(pi):
            tmp = pi + ".tmp.npy"
            af = np.load(pa, mmap_mode="r")
            out = np.lib.format.open_memmap(tmp, mode="w+", dtype=np.float16,
                                            shape=(files.num_institutions, af.shape[1]))
            _mean_into(out, af, files.edge_index("author", "affiliated_with", "institution"),
                       files.num_institutions, dev)
            del out
            os.replace(tmp, pi)
    if comm is not None:
        comm.barrier()
    for p in (pa, pi):
        if not osp.exists(p):
            raise FileNotFoundError(p)
    return {"author": pa, "institution": pi}


def _offsets_from_mapping(mapping: Optional[torch.Tensor], n: int, W: int) -> torch.Tensor:
    """Block offsets from an optional vertex -> rank map (it must already be sorted, i.e.
    the ids renumbered rank-contiguously; ``data.preprocess.node_renumbering`` does that)."""
    if mapping is None:
        return get_vertex_offsets(n, W)
    m = torch.as_tensor(mapping).long()
    if m.numel() != n or (m.numel() > 1 and bool((m[1:] < m[:-1]).any())):
        raise ValueError("rank mapping must cover every vertex and be rank-sorted; renumber "
                         "the vertices first (dgraph_amd.data.preprocess.node_renumbering)")
    off = torch.zeros(W + 1, dtype=torch.long)
    off[1:] = torch.cumsum(torch.bincount(m, minlength=W), 0)
    return off


class DGraph_MAG240M_Dataset(DistributedHeteroGraphDataset):  # noqa: N801 - reference name
    """Per-rank MAG240M: contiguous per-type vertex blocks, five relation plans.

    ``real_features=False`` (the reference's setting: it trains on ``randn(n, 1)`` for all
    three types) draws ``num_features`` random columns per vertex; ``True`` reads this
    rank's rows of the 768-d paper features and of the derived author / institution
    features (generated on first use)."""

    def __init__(self, comm, data_dir: str = "data/MAG240M", comm_plan_only: bool = True,
                 paper_rank_mappings=None, author_rank_mappings=None,
                 institution_rank_mappings=None, cached_comm_plans: Optional[str] = None,
                 real_features: bool = False, num_features: int = 1, seed: int = 0):
        rank, W = comm.get_rank(), comm.get_world_size()
        self.comm = comm
        self.files = files = MAG240MFiles(data_dir)
        counts = [files.num_papers, files.num_authors, files.num_institutions]
        maps = [paper_rank_mappings, author_rank_mappings, institution_rank_mappings]
        offsets = {t: _offsets_from_mapping(maps[t], n, W) for t, n in enumerate(counts)}
        split = {"train": torch.from_numpy(files.get_idx_split("train")).long(),
                 "val": torch.from_numpy(files.get_idx_split("valid")).long(),
                 "test": torch.from_numpy(files.get_idx_split("test-dev")).long()}
        labels = torch.from_numpy(np.nan_to_num(np.asarray(files.paper_label,
                                                           dtype=np.float32))).long()
        feats = []
        if real_features:
            paths = generate_feature_data(files, comm)
            srcs = [files.paper_feat, np.load(paths["author"], mmap_mode="r"),
                    np.load(paths["institution"], mmap_mode="r")]
        g = torch.Generator().manual_seed(seed)
        for t, n in enumerate(counts):
            lo, hi = int(offsets[t][rank]), int(offsets[t][rank + 1])
            if real_features:
                feats.append(torch.from_numpy(np.array(srcs[t][lo:hi], dtype=np.float32)))
            else:
                feats.append(torch.randn(hi - lo, num_features, generator=g))
        self.num_local_papers, self.num_local_authors, self.num_local_institutions = (
            f.shape[0] for f in feats)
        rels = self._relations(files, comm, offsets, rank, W, data_dir, cached_comm_plans)
        super().__init__(rank, W, feats[0].shape[1], files.num_classes, feats, offsets, labels,
                         split, rels)
        for et, r in zip(EDGE_TYPES, rels):  # reference attribute names
            setattr(self, PLAN_KEYS[et], r)

    @staticmethod
    def plan_path(data_dir: str, rank: int, world_size: int) -> str:
        return osp.join(data_dir, f"MAG240M_dataset_rank_{rank}_of_{world_size}_comm_plans.pt")

    @staticmethod
    def _relations(files, comm, offsets, rank, W, data_dir, cached):
        path = cached or DGraph_MAG240M_Dataset.plan_path(data_dir, rank, W)
        # fingerprint of what the plans depend on (sizes, world, rank, per-type ownership):
        # a file written for another partition or world size is rebuilt, not trusted
        meta = torch.cat([torch.tensor([files.num_papers, files.num_authors,
                                        files.num_institutions, W, rank])]
                         + [offsets[t].long() for t in range(3)])
        if osp.exists(path):
            d = torch.load(path, weights_only=True)
            if "_meta" not in d or torch.equal(d["_meta"], meta):
                return [RelationGraph.from_state_dict(d[PLAN_KEYS[et]]) for et in EDGE_TYPES]
            if cached:
                raise ValueError(f"{cached}: plans were built for another partition/world size")
        elif cached:
            raise FileNotFoundError(cached)
        def load(*k):
            return torch.from_numpy(np.array(files.edge_index(*k), dtype=np.int64))

        p2p = load("paper", "cites", "paper")
        p2p = torch.cat([p2p, p2p.flip(0)], dim=1)
        a2p = load("author", "writes", "paper")
        a2i = load("author", "affiliated_with", "institution")
        rel_edges = {(0, 0): p2p, (0, 1): a2p.flip(0), (1, 0): a2p, (1, 2): a2i,
                     (2, 1): a2i.flip(0)}
        group = getattr(comm, "group", None)
        rels = [build_relation_graph(rel_edges[et], et[0], et[1], offsets, rank, W, group)
                for et in EDGE_TYPES]
        d = {PLAN_KEYS[et]: r.state_dict() for et, r in zip(EDGE_TYPES, rels)}
        d["_meta"] = meta
        torch.save(d, path)
        return rels
