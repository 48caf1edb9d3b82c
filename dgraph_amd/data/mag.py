"""MAG240M-shaped heterogeneous graphs, generated on the device, per rank.

Counterpart of the OGB-LSC datasets of the reference (``SyntheticHeterogeneousDataset``,
experiments/OGB-LSC/lsc_datasets/synthetic_dataset.py:38-199; ``DGraph_MAG240M_Dataset``,
MAG240M_dataset.py:116-320) at the scale BASELINE.json names (config 4: MAG240M-shaped
R-GCN on 8 GPUs). The reference builds every relation's plan from the GLOBAL edge lists on
every rank (distributed_graph_dataset.py:113-115, >128 GB host RAM for MAG240M); here each
rank regenerates the edge chunks from a counter-based seed on its GPU and keeps only the
messages that aggregate at vertices it owns, like :mod:`dgraph_amd.data.synthetic`.

Node types: 0 = paper, 1 = author, 2 = institution (contiguous per-rank blocks). Relations
are the reference's ``edge_type = [(0,0), (0,1), (1,0), (1,2), (2,1)]`` = (source type,
destination type): paper->paper (citations, both directions), paper->author and
author->paper (``writes``), author->institution and institution->author (``affiliated``).

Structure: like the homogeneous generator, a fraction ``global_frac`` of the edges has a
uniformly random, hub-skewed endpoint and the rest stay within a window around the
"aligned" position (author ``a`` sits next to paper ``a * P / A``), which is what a
METIS-style co-partitioning of papers and their authors yields.

:func:`build_hetero_partition` returns, for every SOURCE node type, all relations reading
that type stacked by destination rows, with one halo (the union over those relations) and
one send plan — so a layer does ONE halo exchange per source type instead of one per
relation (SURVEY §5.8 "coalesce small per-layer tensors into one grouped exchange").
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from ..ops.csr import CSR, index_dtype_for
from .synthetic import _mix, contiguous_offsets, localize_columns

PAPER, AUTHOR, INSTITUTION = 0, 1, 2
EDGE_TYPES: List[Tuple[int, int]] = [(0, 0), (0, 1), (1, 0), (1, 2), (2, 1)]


@dataclass(frozen=True)
class HeteroShape:
    name: str
    num_nodes: Tuple[int, int, int]    # papers, authors, institutions
    cites: int                          # directed paper->paper pairs (symmetrised)
    writes: int                         # author-paper pairs
    affiliated: int                     # author-institution pairs
    num_features: int
    num_classes: int
    train_frac: float

    def scaled(self, f: float) -> "HeteroShape":
        n = tuple(max(int(v * f), 16) for v in self.num_nodes)
        return HeteroShape(f"{self.name}@{f:g}", n, max(int(self.cites * f), 16),
                           max(int(self.writes * f), 16), max(int(self.affiliated * f), 16),
                           self.num_features, self.num_classes, self.train_frac)

    def messages_per_layer(self) -> int:
        """Directed messages over all five relations (each undirected pair twice)."""
        return 2 * (self.cites + self.writes + self.affiliated)


HETERO_SHAPES = {
    # OGB-LSC MAG240M public sizes; train split 1,112,392 papers
    "mag240m": HeteroShape("mag240m", (121_751_666, 122_383_112, 25_721), 1_297_748_926,
                           386_022_720, 44_592_586, 768, 153, 1_112_392 / 121_751_666),
    # the reference's synthetic default (OGB-LSC/config.py:38-45)
    "synthetic-small": HeteroShape("synthetic-small", (2048, 8192, 256), 2048 * 11,
                                   int(8192 * 3.5), int(8192 * 0.35), 768, 153, 0.7),
}

_CHUNK = 1 << 26


def _edge_chunk(kind: int, shape: HeteroShape, k: int, n: int, seed: int, global_frac: float,
                window: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Chunk ``k`` of edge set ``kind`` (0 cites P-P, 1 writes A-P, 2 affiliated A-I) as
    (u, v) global ids: u in the first type, v in the second."""
    g = torch.Generator(device=device)
    g.manual_seed(_mix(seed, 0x4D4147, kind, k))
    P, A, I = shape.num_nodes
    nu, nv = {0: (P, P), 1: (A, P), 2: (A, I)}[kind]
    u = torch.randint(0, nu, (n,), generator=g, device=device, dtype=torch.int64)
    r = torch.rand(n, generator=g, device=device)
    is_global = torch.rand(n, generator=g, device=device) < global_frac
    hub = (r * r * nv).long().clamp_(max=nv - 1)
    gv = (hub * 2_147_483_629 + 7919) % nv
    # aligned position of u in v's id space, plus a symmetric window offset
    w = max(1, min(window, nv // 2))
    base = u if nu == nv else torch.div(u * nv, nu, rounding_mode="floor")
    lv = (base + ((r * 2 - 1) * w).long()) % nv
    return u, torch.where(is_global, gv, lv)


def _relation_sources(shape: HeteroShape):
    """edge set -> [(relation id, row side, col side)]: side 0 = u, side 1 = v."""
    return {0: [(0, 1, 0), (0, 0, 1)],          # P->P: aggregate at v from u, and at u from v
            1: [(1, 0, 1), (2, 1, 0)],          # P->A at author u from paper v; A->P at v from u
            2: [(3, 1, 0), (4, 0, 1)]}          # A->I at institution v; I->A at author u


def build_relation_csrs(shape: HeteroShape, rank: int, world_size: int, device,
                        seed: int = 0, global_frac: float = 0.05, window: int = 1 << 14,
                        relations: Optional[List[int]] = None):
    """Per-relation CSRs (rows = local destination vertices, GLOBAL source column ids)
    and the per-type offsets. Deterministic and independent of ``world_size``."""
    offs = {t: contiguous_offsets(n, world_size) for t, n in enumerate(shape.num_nodes)}
    want = set(range(5) if relations is None else relations)
    totals = {0: shape.cites, 1: shape.writes, 2: shape.affiliated}
    rows_acc: Dict[int, List[torch.Tensor]] = {r: [] for r in want}
    cols_acc: Dict[int, List[torch.Tensor]] = {r: [] for r in want}
    for kind, rels in _relation_sources(shape).items():
        rels = [x for x in rels if x[0] in want]
        if not rels:
            continue
        E = totals[kind]
        for k in range((E + _CHUNK - 1) // _CHUNK):
            n = min(_CHUNK, E - k * _CHUNK)
            uv = _edge_chunk(kind, shape, k, n, seed, global_frac, window, device)
            for rid, row_side, col_side in rels:
                dt = EDGE_TYPES[rid][1]
                lo, hi = offs[dt][rank], offs[dt][rank + 1]
                rows, cols = uv[row_side], uv[col_side]
                m = (rows >= lo) & (rows < hi)
                rows_acc[rid].append((rows[m] - lo).to(torch.int32))
                cols_acc[rid].append(cols[m].to(torch.int32))
            del uv
    out = {}
    for rid in sorted(want):
        st, dt = EDGE_TYPES[rid]
        L = offs[dt][rank + 1] - offs[dt][rank]
        Ns = shape.num_nodes[st]
        r = torch.cat(rows_acc.pop(rid)).long() if rows_acc.get(rid) else \
            torch.zeros(0, dtype=torch.long, device=device)
        c = torch.cat(cols_acc.pop(rid)).long() if cols_acc.get(rid) else r.clone()
        key, _ = torch.sort(r * Ns + c)  # deterministic (row, col) order, duplicates kept
        del r, c
        r = torch.div(key, Ns, rounding_mode="floor")
        c = (key - r * Ns).to(index_dtype_for(Ns))
        del key
        rowptr = torch.zeros(L + 1, dtype=torch.int64, device=device)
        torch.cumsum(torch.bincount(r, minlength=L), 0, out=rowptr[1:])
        out[rid] = CSR(rowptr, c.contiguous(), Ns)
    return out, offs


def stack_rows(csrs: List[CSR]) -> Tuple[CSR, List[Tuple[int, int]]]:
    """Vertically stack CSRs with the same column space; returns the stacked CSR and each
    part's (row_lo, row_hi)."""
    ranges, rp, cols, base_row, base_nz = [], [], [], 0, 0
    for c in csrs:
        ranges.append((base_row, base_row + c.num_rows))
        rp.append(c.rowptr[(1 if rp else 0):] + base_nz)
        cols.append(c.col)
        base_row += c.num_rows
        base_nz += c.nnz
    rowptr = torch.cat(rp) if rp else torch.zeros(1, dtype=torch.long)
    return CSR(rowptr.contiguous(), torch.cat(cols).contiguous(), csrs[0].num_cols), ranges


def build_hetero_partition(shape: HeteroShape, rank: int, world_size: int, device,
                           seed: int = 0, global_frac: float = 0.05, window: int = 1 << 14,
                           group=None, rehearse: bool = False,
                           relations: Optional[List[int]] = None):
    """Per-source-type stacked relation graphs of ``rank``'s partition.

    Returns ``dict(offsets, sources)``; ``sources[s]`` holds ``csr`` (rows: the stacked
    destination rows of every relation with source type ``s``, cols: [local s | halo s]),
    ``ranges`` {relation id: (row_lo, row_hi)}, ``L`` (local s rows), ``H``, ``halo_gids``,
    ``send_local_idx``, ``send_splits``, ``recv_splits``. Collective over ``group`` when
    ``world_size > 1`` (unless ``rehearse``: loopback send plan of the right size).
    """
    from ..plan.pattern import _alltoall_counts, _alltoallv_ids

    rels, offs = build_relation_csrs(shape, rank, world_size, device, seed, global_frac,
                                     window, relations)
    sources = {}
    for s in range(3):
        rids = [r for r in sorted(rels) if EDGE_TYPES[r][0] == s]
        if not rids:
            continue
        csr_g, rr = stack_rows([rels.pop(r) for r in rids])
        ranges = dict(zip(rids, rr))
        o = offs[s]
        L = o[rank + 1] - o[rank]
        if world_size == 1:
            csr_g.num_cols = L
            sources[s] = dict(csr=csr_g, ranges=ranges, L=L, H=0,
                              halo_gids=csr_g.col[:0].long(),
                              send_local_idx=torch.zeros(0, dtype=torch.int32, device=device),
                              send_splits=[0], recv_splits=[0])
            continue
        csr, halo, recv_splits = localize_columns(csr_g, rank, o)
        del csr_g
        if rehearse:
            send_splits = list(recv_splits)
            n = sum(send_splits)
            sli = (torch.arange(n, device=device, dtype=torch.long) * 7919 % max(L, 1)).to(
                index_dtype_for(L))
        else:
            req = torch.tensor(recv_splits, dtype=torch.long, device=device)
            send_splits = [int(v) for v in _alltoall_counts(req, group).tolist()]
            wanted = _alltoallv_ids(halo, recv_splits, send_splits, group)
            sli = (wanted - o[rank]).to(index_dtype_for(L))
        sources[s] = dict(csr=csr, ranges=ranges, L=L, H=int(halo.numel()), halo_gids=halo,
                          send_local_idx=sli, send_splits=send_splits,
                          recv_splits=recv_splits)
    return dict(offsets=offs, sources=sources)


def hetero_node_data(shape: HeteroShape, rank: int, offsets, device, seed: int = 0,
                     dtype=torch.bfloat16, feature_types=(0, 1, 2), alloc=None):
    """Random features per node type ([L_t, F], seeded per global vertex chunk so values do
    not depend on W), paper labels and the paper train mask. ``alloc(type, shape, dtype)`` places
    the feature tensors (e.g. on the symmetric heap for one-sided remote gets)."""
    C = 1 << 20
    feats = {}
    for t in feature_types:
        lo, hi = offsets[t][rank], offsets[t][rank + 1]
        x = alloc(t, (hi - lo, shape.num_features), dtype) if alloc is not None else \
            torch.empty(hi - lo, shape.num_features, device=device, dtype=dtype)
        g = torch.Generator(device=device)
        for c in range(lo // C, (hi + C - 1) // C):
            a, b = c * C, min((c + 1) * C, shape.num_nodes[t])
            g.manual_seed(_mix(seed, 0x66656174, t, c))
            xc = torch.randn(b - a, shape.num_features, generator=g, device=device)
            s, e = max(a, lo), min(b, hi)
            x[s - lo:e - lo] = xc[s - a:e - a].to(dtype)
            del xc
        feats[t] = x
    lo, hi = offsets[PAPER][rank], offsets[PAPER][rank + 1]
    y = torch.empty(hi - lo, dtype=torch.int64, device=device)
    train = torch.empty(hi - lo, dtype=torch.bool, device=device)
    g = torch.Generator(device=device)
    for c in range(lo // C, (hi + C - 1) // C):
        a, b = c * C, min((c + 1) * C, shape.num_nodes[PAPER])
        g.manual_seed(_mix(seed, 0x6C61626C, c))
        yc = torch.randint(0, shape.num_classes, (b - a,), generator=g, device=device)
        tc = torch.rand(b - a, generator=g, device=device) < shape.train_frac
        s, e = max(a, lo), min(b, hi)
        y[s - lo:e - lo] = yc[s - a:e - a]
        train[s - lo:e - lo] = tc[s - a:e - a]
    return feats, y, train
