"""Relational GCN for heterogeneous graphs (BASELINE config 4: MAG240M-shaped R-GCN).

The reference ships only an RGAT for OGB-LSC (experiments/OGB-LSC/RGAT.py:271-382); this
is the R-GCN (mean-aggregating relational graph conv, the OGB-LSC "R-GraphSAGE" baseline)
with the same layer skeleton — per-layer skip ``Linear`` shared by all node types, one
convolution per relation, synchronised BatchNorm, ReLU, dropout, MLP head on the target
type — so it plugs into the same trainer:

    h_d^{l+1} = dropout(relu(BN( skip_l(h_d^l) + sum_{r: s->d} mean_{j in N_r(i)} h_s^l[j] W_r^l )))

Execution paths:

* :class:`HeteroGraph`, fp32 (the reference's precision) — :meth:`_forward_hetero_lean`:
  transform-first at every layer, BN'd activations recomputed in backward instead of saved,
  relation aggregations added in place into the destinations' pre-activations, GEMMs on the
  exact-f32 MFMA kernels; fits rank 1 of the 8-way MAG240M partition on one GPU.
* :class:`HeteroGraph`, bf16 autocast (``dgraph_amd.parallel.hetero_graph``; built by
  ``dgraph_amd.data.mag.build_hetero_partition``) — the MI355X hot path. Layer 0 is
  transform-first: ONE GEMM per source type ``X_s [W_r1 | W_r2 ...]`` on the local rows
  and on the halo feature rows fetched once (one-sided heap get, or one all-to-all-v), then
  per-relation SpMMs over column slices — no communication at all in layer 0, forward or
  backward. Later layers aggregate first with one overlapped halo exchange per source
  type. Only the (layer, type) pairs that reach the loss are computed (a 2-layer model
  never touches the author->institution relation, and its last layer updates papers only).
* :class:`dgraph_amd.data.hetero.RelationGraph` lists (the RGAT dataset objects) — the
  per-relation halo-exchange path, for API parity with ``CommAwareRGAT``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.act_linear import act_linears
from ..ops.aggregate import aggregate
from ..ops.dense import linear as _dense_linear
from ..ops.dense import linear_sum
from ..parallel.hetero_graph import SourceGraph, source_aggregate, source_aggregate_into
from .norm import DistributedBatchNorm1D


@dataclass
class HeteroGraph:
    """One rank's view: ``sources[s]`` = :class:`SourceGraph` of source type ``s``;
    ``num_local[t]`` = owned vertices of type ``t``."""

    sources: Dict[int, SourceGraph]
    num_local: Dict[int, int]
    edge_types: List[Tuple[int, int]]
    extra: dict = field(default_factory=dict)

    @staticmethod
    def from_partition(part: dict, edge_types, group=None, overlap: bool = True,
                       rank: int = 0) -> "HeteroGraph":
        offs = part["offsets"]
        srcs = {s: SourceGraph.from_partition(d, group, overlap, src_offsets=offs[s])
                for s, d in part["sources"].items()}
        nl = {t: offs[t][rank + 1] - offs[t][rank] for t in offs}
        return HeteroGraph(srcs, nl, list(edge_types))


def layer_plan(edge_types: Sequence[Tuple[int, int]], num_layers: int, target: int = 0,
               available: Optional[Sequence[int]] = None):
    """(types computed, relations used) per layer, pruned backwards from the target type."""
    need = [set() for _ in range(num_layers)]
    rels = [[] for _ in range(num_layers)]
    want = {target}
    for l in range(num_layers - 1, -1, -1):
        need[l] = set(want)
        rels[l] = [r for r, (s, d) in enumerate(edge_types)
                   if d in want and (available is None or r in available)]
        want = set(want) | {edge_types[r][0] for r in rels[l]}
    return need, rels


class CommAwareRGCN(nn.Module):
    def __init__(self, in_channels: int, hidden_channels: int, out_channels: int,
                 num_relations: int, num_layers: int = 2, dropout: float = 0.5,
                 edge_types: Optional[Sequence[Tuple[int, int]]] = None, comm=None,
                 target_type: int = 0, bn_group=None, num_node_types: int = 3):
        super().__init__()
        self.num_layers, self.dropout, self.comm = num_layers, dropout, comm
        self.hidden = hidden_channels
        self.edge_types = list(edge_types) if edge_types is not None else None
        self.target = target_type
        self.num_node_types = num_node_types
        self.lean: Optional[bool] = None  # None: by the compute dtype (see forward)
        self.static_halo: Optional[bool] = None  # lean path; None: by memory
        self.convs = nn.ModuleList()
        self.skips = nn.ModuleList()
        for i in range(num_layers):
            cin = in_channels if i == 0 else hidden_channels
            self.convs.append(nn.ModuleList([nn.Linear(cin, hidden_channels, bias=False)
                                             for _ in range(num_relations)]))
            self.skips.append(nn.Linear(cin, hidden_channels))
        self.bns = nn.ModuleList([DistributedBatchNorm1D(hidden_channels, recompute=True,
                                                         group=bn_group)
                                  for _ in range(num_layers)])
        self.mlp = nn.Sequential(
            nn.Linear(hidden_channels, hidden_channels),
            DistributedBatchNorm1D(hidden_channels, recompute=True, group=bn_group),
            nn.ReLU(inplace=True),
            nn.Dropout(dropout),
            nn.Linear(hidden_channels, out_channels),
        )

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _lin(mod: nn.Linear, x: torch.Tensor) -> torch.Tensor:
        # tall-skinny-aware backward: split-K weight gradient, native bias column sum
        return _dense_linear(x, mod.weight, mod.bias)

    def _head(self, h: torch.Tensor) -> torch.Tensor:
        lin1, bn, _, drop, lin2 = self.mlp
        t = bn(self._lin(lin1, h), relu=True, dropout=drop.p)  # BN + ReLU + dropout fused
        return self._lin(lin2, t)

    def _finish(self, l: int, t: torch.Tensor) -> torch.Tensor:
        # BN + ReLU + dropout in one pass (native kernels on GPU; the dropout mask is
        # regenerated from a seed in backward: no mask tensor, no masked-scale pass)
        return self.bns[l](t, relu=True, dropout=self.dropout)

    def forward(self, xs, graph, edge_types=None) -> torch.Tensor:
        """``forward(xs, HeteroGraph)`` (hot path), or the RelationGraph path with either
        argument order: ``(xs, graphs, edge_types)`` or RGAT's ``(xs, edge_types, graphs)``.

        HeteroGraph inputs computed in fp32 (the reference's precision) take the
        memory-lean path (:meth:`_forward_hetero_lean`); under bf16 autocast the
        aggregate-first path with the bf16 MFMA dual GEMM (:meth:`_forward_hetero`)."""
        if isinstance(graph, HeteroGraph):
            x0 = next(iter(xs.values()))
            lean = self.lean if self.lean is not None else (
                x0.dtype == torch.float32 and not (torch.is_autocast_enabled() and x0.is_cuda))
            if lean:
                return self._forward_hetero_lean(xs, graph)
            return self._forward_hetero(xs, graph)
        if edge_types is not None and len(graph) and isinstance(graph[0], tuple):
            graph, edge_types = edge_types, graph
        return self._forward_relations(xs, edge_types, graph)

    # ------------------------------------------------------------------ hot path
    def _forward_hetero(self, xs: Dict[int, torch.Tensor], g: HeteroGraph) -> torch.Tensor:
        ets = g.edge_types
        avail = [r for s in g.sources.values() for r in s.ranges]
        need, rels = layer_plan(ets, self.num_layers, self.target, avail)
        h = dict(xs)
        for l in range(self.num_layers):
            tmp = {t: self._lin(self.skips[l], h[t]) for t in sorted(need[l])} if l == 0 else {}
            # layers > 0: skip + one linear per relation summed by ONE fused op per
            # destination type (the MFMA dual GEMM chains the running sum: no per-term
            # outputs, no elementwise adds)
            terms = {t: [(h[t], self.skips[l].weight)] for t in sorted(need[l])} if l else {}
            by_src: Dict[int, List[int]] = {}
            for r in rels[l]:
                by_src.setdefault(ets[r][0], []).append(r)
            for s, rs in sorted(by_src.items()):
                sg = g.sources[s]
                if l == 0:
                    # transform-first: one GEMM over [W_r1 | W_r2 ...], static halo rows
                    W = torch.cat([self.convs[0][r].weight for r in rs], 0)
                    z = _dense_linear(h[s], W)
                    xh = sg.static_halo(xs[s])
                    zh = _dense_linear(xh, W) if xh is not None else None
                    C = self.hidden
                    spec = [(r, i * C, (i + 1) * C) for i, r in enumerate(rs)]
                    outs = source_aggregate(z, sg, spec, static_halo=zh) if zh is not None \
                        else source_aggregate(z, sg, spec)
                    for r, o in zip(rs, outs):
                        d = ets[r][1]
                        tmp[d] = tmp[d].add_(o.to(tmp[d].dtype))  # linear outputs are not saved
                else:
                    spec = [(r, 0, h[s].shape[1]) for r in rs]
                    outs = source_aggregate(h[s], sg, spec)
                    for r, o in zip(rs, outs):
                        terms[ets[r][1]].append((o, self.convs[l][r].weight))
            for t, tl in terms.items():
                tmp[t] = linear_sum(tl, self.skips[l].bias)
            h = {t: self._finish(l, v) for t, v in tmp.items()}
        return self._head(h[self.target])

    def _keep_static_halo(self, xs: Dict[int, torch.Tensor], g: HeteroGraph) -> bool:
        """Keep the layer-0 feature halo rows for the whole run (fetched once, no layer-0
        communication) unless they would take more than ``STATIC_HALO_FRAC`` of the
        device; then the transformed rows of every relation are exchanged per step
        instead (256 instead of 768 columns, and nothing resident)."""
        if self.static_halo is not None:
            return bool(self.static_halo)
        nbytes = sum(sg.H * xs[s].shape[1] * xs[s].element_size()
                     for s, sg in g.sources.items() if s in xs)
        x0 = next(iter(xs.values()))
        if not x0.is_cuda or nbytes == 0:
            return True
        total = torch.cuda.get_device_properties(x0.device).total_memory
        return nbytes <= self.STATIC_HALO_FRAC * total

    STATIC_HALO_FRAC = 0.08

    def _forward_hetero_lean(self, xs: Dict[int, torch.Tensor], g: HeteroGraph) -> torch.Tensor:
        """Transform-first at EVERY layer, BN'd activations recomputed instead of stored:

            pre_t^l = skip_l(h_t) + sum_{r: s->t} mean_r(h_s W_r^l),  h = act(BN(pre^{l-1}))

        per source type ONE :func:`~dgraph_amd.ops.act_linears` call builds ``act(BN(pre_s))``
        transiently and runs the skip GEMM (straight into ``pre_s``, bias fused) and one GEMM
        per relation; each relation's aggregation then adds into its destination's ``pre``
        in place, exchanging that relation's transformed halo rows (one [H, hidden] buffer
        live at a time). Saved per step: the inputs, one ``pre`` per (layer, type) and the
        head's hidden pre-activation — no BN output, aggregate or relation output (the
        aggregate-first path saves each of those: 274 GB at fp32 on one GPU's 1/8 MAG240M
        share, profiles/r04/rgcn_fp32_eighth.json). Layer 0's feature halo rows are kept
        (fetched once) when :meth:`_keep_static_halo` allows. Same math as
        :meth:`_forward_hetero`."""
        ets = g.edge_types
        avail = [r for s in g.sources.values() for r in s.ranges]
        need, rels = layer_plan(ets, self.num_layers, self.target, avail)
        keep_halo = self._keep_static_halo(xs, g)
        pre: Dict[int, torch.Tensor] = {}
        for l in range(self.num_layers):
            by_src: Dict[int, List[int]] = {}
            for r in rels[l]:
                by_src.setdefault(ets[r][0], []).append(r)
            new: Dict[int, torch.Tensor] = {}
            zs = []
            for s in sorted(set(need[l]) | set(by_src)):
                rs = by_src.get(s, [])
                skip = s in need[l]
                Ws = ([self.skips[l].weight] if skip else []) + \
                    [self.convs[l][r].weight for r in rs]
                inp = xs[s] if l == 0 else pre[s]
                bn = self.bns[l - 1] if l else None
                outs = act_linears(inp, Ws, self.skips[l].bias if skip else None,
                                   bn=bn, relu=l > 0, dropout=self.dropout if l else 0.0)
                if skip:
                    new[s] = outs[0]
                zr = outs[1:] if skip else outs
                zh = [None] * len(rs)
                if l == 0 and keep_halo:
                    # read-only features: halo rows fetched once, transformed here
                    xh = g.sources[s].static_halo(xs[s])
                    if xh is not None:
                        zh = act_linears(xh, Ws[len(Ws) - len(rs):])
                zs += [(s, r, z, h) for r, z, h in zip(rs, zr, zh)]
            while zs:  # each relation output is released right after its aggregation
                s, r, z, zh = zs.pop(0)
                d = ets[r][1]
                new[d] = source_aggregate_into(z, g.sources[s], [(r, 0, z.shape[1])],
                                               [new[d]], static_halo=zh)[0]
                del z, zh
            pre = new
        lin1, bn, _, drop, lin2 = self.mlp
        t = self.target
        p1 = act_linears(pre[t], [lin1.weight], lin1.bias, bn=self.bns[self.num_layers - 1],
                         relu=True, dropout=self.dropout)[0]
        return act_linears(p1, [lin2.weight], lin2.bias, bn=bn, relu=True,
                           dropout=drop.p)[0]

    # ------------------------------------------------------------------ RelationGraph path
    def _forward_relations(self, xs: List[torch.Tensor], edge_types, graphs) -> torch.Tensor:
        from ..parallel.halo import HaloExchange
        import torch.distributed as dist

        ets = list(edge_types)
        W = self.comm.get_world_size() if self.comm is not None else (
            dist.get_world_size() if dist.is_initialized() else 1)
        need, rels = layer_plan(ets, self.num_layers, self.target)
        h = list(xs)
        halo = HaloExchange(self.comm) if W > 1 else None
        for l in range(self.num_layers):
            tmp = {t: self.skips[l](h[t]) for t in sorted(need[l])}
            for r in rels[l]:
                s, d = ets[r]
                g = graphs[r]
                xs_all = h[s]
                if halo is not None:
                    xs_all = torch.cat([xs_all, halo(h[s], g.pattern)], 0)
                agg = aggregate(xs_all, g.csr, reduce="mean")
                tmp[d] = tmp[d] + self.convs[l][r](agg)
            h = dict(h) if isinstance(h, dict) else {i: v for i, v in enumerate(h)}
            h.update({t: self._finish(l, v) for t, v in tmp.items()})
        return self._head(h[self.target])
