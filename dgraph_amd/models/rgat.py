"""Graph attention for heterogeneous graphs (experiments/OGB-LSC/RGAT.py:44-382).

``CommAwareGAT`` computes, for every destination vertex ``i`` of one relation,
``out_i = sum_j alpha_ij h_j (+ W_res x_i) (+ b)`` with ``h = W x`` and
``alpha_ij = softmax_j(leaky_relu(a . [h_i || h_j] + c))``.

MI355X formulation (``_forward_graph``, used with a :class:`RelationGraph`):

* the attention logit is split over the concatenation, ``a . [h_i || h_j] =
  s_dst[i] + s_src[j]`` — two vertex-level reductions instead of an ``E x 2F`` concat and
  an ``E``-row GEMV;
* ONE halo exchange per relation moves ``[h_j || s_src_j]`` rows of remote sources;
* per-edge work is three native kernels: logits (``gather_add_act``, leaky-ReLU), a
  max-subtracted edge softmax over each destination's CSR segment (the reference's
  ``exp`` had no max subtraction, RGAT.py:154) and the edge-weighted multi-head SpMM;
  no atomics, no per-edge feature tensors.

``heads`` splits the channels into ``heads`` attention heads (the reference accepted and
ignored it). The reference's plan-based (G2, ``NCCLEdgeConditionedGraphCommPlan``) and
index-based (G1 COO) forwards are kept for API parity.

``CommAwareRGAT`` runs ALL relations of every layer (the reference broke out after the
first relation, RGAT.py:357-358; ``relations="first"`` restores that behaviour).

Lean fp32 path (``CommAwareRGAT.forward(xs, HeteroGraph)``, :meth:`CommAwareRGAT.
_forward_hetero_lean`): the R-GCN treatment (models/rgcn.py) — transform-first with the
exact-f32 MFMA linears, ONE :func:`~dgraph_amd.ops.act_linear.act_linears` call per source
type builds ``act(BN(pre))`` transiently and runs every GEMM that reads it (the skip and
all residual transforms of its destination relations folded into ONE weight, each
relation's ``W_r``, and each relation's destination-score projection
``V_r = a_dst W_r`` so ``h_i`` is never formed); each relation's attention is the fused
kernel of ``ops/gat.py`` added in place into its destination's pre-activation, with its halo
rows exchanged by one all-to-all-v (layer 0: the kept halo feature rows are transformed
locally, no exchange) and read as a second source (no ``torch.cat``); BN / ReLU / dropout are
recomputed in backward instead of stored.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops.aggregate import aggregate, edge_softmax
from ..ops.act_linear import act_linears
from ..ops.edge_mlp import edge_pre_activation
from .norm import DistributedBatchNorm1D


def _world(comm) -> int:
    if comm is not None:
        return comm.get_world_size()
    return dist.get_world_size() if dist.is_initialized() else 1


class ConvLayer(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Linear(in_channels, out_channels)
        self.act = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.act(self.conv(x))


class CommAwareGAT(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, comm=None, heads: int = 1,
                 bias: bool = True, residual: bool = False, hetero: bool = False):
        super().__init__()
        if out_channels % heads:
            raise ValueError("out_channels must be divisible by heads")
        self.conv1 = nn.Linear(in_channels, out_channels, bias=False)
        self.comm = comm
        self.project_message = nn.Linear(2 * out_channels, heads)
        self.leaky_relu = nn.LeakyReLU(0.2, inplace=False)
        self.residual = residual
        self.heads = heads
        self.hetero = hetero
        self.out_channels = out_channels
        if residual:
            self.res_net = nn.Linear(in_channels, out_channels, bias=False)
        if bias:
            self.bias = nn.Parameter(torch.zeros(out_channels))
        else:
            self.register_parameter("bias", None)
        self._halo = None

    # ------------------------------------------------------------------ dispatch
    def forward(self, x, comm_plan=None, *, x_j=None, graph=None, edge_index=None,
                rank_mapping=None, src_gather_cache=None, dest_gather_cache=None,
                dest_scatter_cache=None):
        from ..data.hetero import RelationGraph

        if isinstance(comm_plan, RelationGraph):
            graph, comm_plan = comm_plan, None
        if graph is not None:
            return self._forward_graph(x, graph, x_j)
        if comm_plan is not None:
            return self._forward_comm_plan(x, comm_plan, x_j=x_j)
        return self._forward_coo(x, edge_index, rank_mapping, x_j, src_gather_cache,
                                 dest_gather_cache, dest_scatter_cache)

    def _head_scores(self, h: torch.Tensor, part: int) -> torch.Tensor:
        """``s[:, k] = h[:, head k] . a_k`` with ``a_k`` the head-k block of the
        destination (part 0) or source (part 1) half of ``project_message``."""
        H, C = self.heads, self.out_channels
        D = C // H
        W = self.project_message.weight[:, part * C:(part + 1) * C]  # [H, C]
        if H == 1:
            return h @ W.t()
        blocks = torch.stack([W[k, k * D:(k + 1) * D] for k in range(H)])  # [H, D]
        return (h.view(-1, H, D) * blocks.to(h.dtype)).sum(-1)

    def _apply_res_and_bias(self, out, x):
        if self.residual:
            out = out + self.res_net(x)
        if self.bias is not None:
            out = out + self.bias
        return out

    # ------------------------------------------------------------------ fast path
    def _forward_graph(self, x, graph, x_j=None):
        C, H = self.out_channels, self.heads
        h = self.conv1(x)
        hj = self.conv1(x_j) if (self.hetero and x_j is not None) else h
        s_dst = self._head_scores(h, 0) + self.project_message.bias.to(h.dtype)
        s_src = self._head_scores(hj, 1)
        payload = torch.cat([hj, s_src.to(hj.dtype)], dim=1)
        if _world(self.comm) > 1:  # collective on every rank of the relation's group
            from ..parallel.halo import HaloExchange

            if self._halo is None:
                self._halo = HaloExchange(self.comm)
            halo = self._halo(payload, graph.pattern)
            payload = torch.cat([payload, halo], dim=0)
        hj_all, ssrc_all = payload[:, :C], payload[:, C:]
        logits = edge_pre_activation(None, s_dst.to(payload.dtype), ssrc_all,
                                     graph.row_map(), graph.col_map(), act="leaky_relu")
        # softmax statistics in fp32 (fp64 inputs stay fp64)
        alpha = edge_softmax(logits if logits.dtype == torch.float64 else logits.float(),
                             graph.csr)
        out = aggregate(hj_all, graph.csr, edge_weight=alpha, heads=H)
        return self._apply_res_and_bias(out, x)

    # ------------------------------------------------------------------ reference paths
    def _process_messages(self, h, h_j):
        """``exp(leaky_relu(a . [h_i || h_j] + c))`` per head (the reference's unnormalised
        numerator, RGAT.py:146-156), with the same per-head score blocks as the fast path
        (identical to the reference's ``Linear(2C, 1)`` at one head)."""
        s = self._head_scores(h, 0) + self._head_scores(h_j, 1) + \
            self.project_message.bias.to(h.dtype)
        return torch.exp(self.leaky_relu(s))

    def _calc_attention_messages(self, neighbor_features, numerator, denominator):
        alpha = numerator / (denominator + 1e-16)
        H = self.heads
        nf = neighbor_features.reshape(*neighbor_features.shape[:-1], H, -1)
        return (nf * alpha.unsqueeze(-1)).reshape(neighbor_features.shape)

    def _forward_comm_plan(self, x, comm_plan, x_j=None):
        """G2 plan path (RGAT.py:171-201), with its five collectives per relation-layer
        (two gathers, scatter + gather of the denominator, scatter of the messages) cut to
        TWO: one grouped all-to-all-v carries both endpoint gathers
        (:func:`~dgraph_amd.parallel.plan_ops.plan_gather_grouped`), and one scatter carries
        ``[num * h_j | num]`` so every destination divides its own message sum by its own
        denominator — ``sum_j num_ij h_j / (den_i + 1e-16)`` is the reference's
        ``sum_j (num_ij / (den_i + 1e-16)) h_j``. Backward: the adjoints, two more."""
        from ..parallel.plan_ops import plan_gather_grouped, plan_scatter

        h = self.conv1(x)
        src_plan = comm_plan.source_graph_plan
        if self.hetero:
            h_j = self.conv1(x_j)
            dst_plan = comm_plan.dest_graph_plan
        else:
            h_j, dst_plan = h, src_plan
        group = getattr(self.comm, "group", None) if self.comm is not None else None
        h_i, h_j = plan_gather_grouped([h, h_j], [dst_plan, src_plan], group)
        num = self._process_messages(h_i, h_j)  # [E, heads]
        C, H = self.out_channels, self.heads
        msg = (h_j.view(-1, H, C // H) * num.unsqueeze(-1).to(h_j.dtype)).reshape(-1, C)
        agg = plan_scatter(torch.cat([msg, num.to(msg.dtype)], dim=1), dst_plan, group)
        den = agg[:, C:] + 1e-16
        out = (agg[:, :C].view(-1, H, C // H) / den.unsqueeze(-1)).reshape(-1, C)
        return self._apply_res_and_bias(out, x)

    def _forward_coo(self, x, edge_index, rank_mapping, x_j=None, src_gather_cache=None,
                     dest_gather_cache=None, dest_scatter_cache=None):
        """G1 index path (RGAT.py:208-268)."""
        h = self.conv1(x)
        h_j = self.conv1(x_j) if self.hetero else h
        src_idx, dst_idx = edge_index[:, 0, :], edge_index[:, 1, :]
        src_rm = torch.cat([rank_mapping[0].unsqueeze(0), rank_mapping[0].unsqueeze(0)], 0)
        dst_rm = torch.cat([rank_mapping[0].unsqueeze(0), rank_mapping[1].unsqueeze(0)], 0)
        h_i = self.comm.gather(h, dst_idx, dst_rm, cache=dest_gather_cache)
        h_j = self.comm.gather(h_j, src_idx, src_rm, cache=src_gather_cache)
        num = self._process_messages(h_i, h_j)
        den = self.comm.scatter(num, dst_idx, dst_rm, h.size(-2), cache=dest_scatter_cache)
        den = self.comm.gather(den, src_idx, src_rm, cache=dest_gather_cache)
        out = self.comm.scatter(self._calc_attention_messages(h_j, num, den), dst_idx, dst_rm,
                                h.size(-2), cache=dest_scatter_cache)
        return self._apply_res_and_bias(out, x)


class CommAwareRGAT(nn.Module):
    def __init__(self, in_channels, out_channels, hidden_channels, num_relations, num_layers,
                 heads, comm=None, dropout: float = 0.5, relations: str = "all",
                 num_node_types: int = 3, bn_group=None):
        super().__init__()
        self.num_layers, self.dropout, self.comm = num_layers, dropout, comm
        self.num_relations = num_relations
        self.relations = relations
        self.layers = nn.ModuleList()
        for i in range(num_layers):
            cin = in_channels if i == 0 else hidden_channels
            self.layers.append(nn.ModuleList([
                CommAwareGAT(cin, hidden_channels, heads=heads, bias=True, residual=True,
                             comm=comm, hetero=True) for _ in range(num_relations)]))
        self.bn_layers = nn.ModuleList([
            DistributedBatchNorm1D(hidden_channels, recompute=True, group=bn_group)
            for _ in range(num_layers)])
        self.skip_layers = nn.ModuleList(
            [nn.Linear(in_channels, hidden_channels)]
            + [nn.Linear(hidden_channels, hidden_channels) for _ in range(num_layers - 1)])
        self.num_node_types = num_node_types
        self.mlp = nn.Sequential(
            nn.Linear(hidden_channels, hidden_channels),
            DistributedBatchNorm1D(hidden_channels, recompute=True, group=bn_group),
            nn.ReLU(inplace=True),
            nn.Dropout(dropout),
            nn.Linear(hidden_channels, out_channels),
        )
        self.static_halo: Optional[bool] = None  # lean path; None: by memory (R-GCN's rule)
        # lean path: layer-0 z rebuilt in backward instead of saved — None (auto): when the
        # graph has halos (W > 1: their exchanged rows add to the step's memory; one GPU's
        # 1/8 MAG240M share fits without, 1542 vs 1666 ms per step with)
        self.remake_layer0: Optional[bool] = None

    STATIC_HALO_FRAC = 0.08

    def forward(self, xs, edge_types, graphs=None) -> torch.Tensor:
        """``forward(xs, edge_types, graphs)`` over per-relation RelationGraphs (API of the
        reference), or ``forward(xs, HeteroGraph)`` — the lean fp32 path."""
        from .rgcn import HeteroGraph

        if isinstance(edge_types, HeteroGraph):
            return self._forward_hetero_lean(xs, edge_types)
        assert len(edge_types) == len(graphs)
        outs = list(xs)
        for i in range(self.num_layers):
            tmp = [self.skip_layers[i](o) for o in outs]
            for j, (et, g) in enumerate(zip(edge_types, graphs)):
                if self.relations == "first" and j > 0:
                    break
                s, d = et
                tmp[d] = tmp[d] + self.layers[i][j](outs[d], g, x_j=outs[s])
            outs = []
            for t in tmp:
                t = torch.relu(self.bn_layers[i](t))
                outs.append(nn.functional.dropout(t, self.dropout, self.training))
        return self.mlp(outs[0])

    # ------------------------------------------------------------------ lean fp32 path
    @staticmethod
    def _att_vectors(conv: CommAwareGAT):
        """(a_dst, a_src) as [heads, D] (per-head blocks of ``project_message``)."""
        H, C = conv.heads, conv.out_channels
        D = C // H
        W = conv.project_message.weight
        a_dst = torch.stack([W[k, k * D:(k + 1) * D] for k in range(H)])
        a_src = torch.stack([W[k, C + k * D:C + (k + 1) * D] for k in range(H)])
        return a_dst, a_src

    def _patterns(self, g) -> Dict[int, "object"]:
        from ..ops.gat import GatPattern

        pats = g.extra.get("gat_patterns")
        if pats is None:
            pats = {}
            for s, sg in g.sources.items():
                for rid in sg.ranges:
                    pats[rid] = GatPattern.merged(sg.part("interior", rid),
                                                  sg.part("halo", rid) if sg.halo is not None
                                                  else None, sg.Ls)
            g.extra["gat_patterns"] = pats
        return pats

    def _forward_hetero_lean(self, xs: Dict[int, torch.Tensor], g) -> torch.Tensor:
        """Transform-first at every layer, activations recomputed in backward:

            pre_t^l = x W_t'^T + b_t' + sum_{r: s->t} att_r(z_r = h_s W_r^T, sd_r = h_t V_r^T)

        with ``W_t' = skip_l + sum_{r->t} res_net_r`` and ``b_t' = skip bias + sum_{r->t}
        bias_r`` (one GEMM instead of 1 + |relations into t|: the skip and residual
        transforms read the same input), ``V_r[k] = a_dst[k] W_r[head k rows]`` and ``att_r``
        the fused relation attention (ops/gat.py) added in place into ``pre_t``."""
        from ..ops.gat import gat_relation_into
        from .rgcn import layer_plan

        ets = g.edge_types
        avail = [r for s in g.sources.values() for r in s.ranges]
        need, rels = layer_plan(ets, self.num_layers, 0, avail)
        pats = self._patterns(g)
        from .rgcn import CommAwareRGCN

        # layer 0's feature halo rows kept (fetched once, transformed locally every step)
        # unless they would take more than STATIC_HALO_FRAC of the device; then each
        # relation's transformed halo rows are exchanged per step like a hidden layer's
        # (256 instead of 768 columns, nothing resident: a W=8 MAG240M rank's feature halo
        # is ~48 GB)
        keep_halo = CommAwareRGCN._keep_static_halo(self, xs, g)
        remake0 = self.remake_layer0 if self.remake_layer0 is not None else any(
            sg.halo is not None for sg in g.sources.values())
        pre: Dict[int, torch.Tensor] = {}
        for l in range(self.num_layers):
            convs = self.layers[l]
            by_src: Dict[int, List[int]] = {}
            by_dst: Dict[int, List[int]] = {}
            for r in rels[l]:
                by_src.setdefault(ets[r][0], []).append(r)
                by_dst.setdefault(ets[r][1], []).append(r)
            new: Dict[int, torch.Tensor] = {}
            sds: Dict[int, torch.Tensor] = {}
            work = []
            for s in sorted(set(need[l]) | set(by_src)):
                rs_src = by_src.get(s, [])
                rs_dst = by_dst.get(s, []) if s in need[l] else []
                skip = s in need[l]
                Ws, bias = [], None
                if skip:
                    W = self.skip_layers[l].weight
                    b = self.skip_layers[l].bias
                    for r in rs_dst:
                        W = W + convs[r].res_net.weight
                        if convs[r].bias is not None:
                            b = b + convs[r].bias
                    Ws.append(W)
                    bias = b
                Ws += [convs[r].conv1.weight for r in rs_src]
                vs = []
                for r in rs_dst:
                    c = convs[r]
                    a_dst, _ = self._att_vectors(c)
                    Hh, D = a_dst.shape
                    vs.append(torch.einsum("kd,kdc->kc", a_dst,
                                           c.conv1.weight.view(Hh, D, -1)))
                Ws += vs
                inp = xs[s] if l == 0 else pre[s]
                bn = self.bn_layers[l - 1] if l else None
                outs = act_linears(inp, Ws, bias, bn=bn, relu=l > 0,
                                   dropout=self.dropout if l else 0.0)
                k = 0
                if skip:
                    new[s] = outs[0]
                    k = 1
                zs = outs[k:k + len(rs_src)]
                for r, o in zip(rs_dst, outs[k + len(rs_src):]):
                    sds[r] = o + convs[r].project_message.bias
                zh = [None] * len(rs_src)
                xh = None
                if l == 0 and keep_halo:
                    # read-only features: halo rows fetched once, transformed here
                    xh = g.sources[s].static_halo(xs[s])
                    if xh is not None:
                        zh = act_linears(xh, [convs[r].conv1.weight for r in rs_src])
                # layer 0: z = x W_r^T is rebuilt in backward from the resident features
                # rather than kept (saves [rows, hidden] per relation: 47 GB on one GPU's
                # 1/8 MAG240M share)
                rem = [((xs[s], convs[r].conv1.weight) + ((xh,) if xh is not None else ()))
                       if (l == 0 and remake0) else None for r in rs_src]
                work += [(s, r, z, h, q) for r, z, h, q in zip(rs_src, zs, zh, rem)]
            while work:  # each relation's transformed rows released after its attention
                s, r, z, zh, rem = work.pop(0)
                d = ets[r][1]
                _, a_src = self._att_vectors(convs[r])
                sg = g.sources[s]
                new[d] = gat_relation_into(z, sds.pop(r), a_src, new[d], pats[r],
                                           sg=sg if zh is None else None, zh_static=zh,
                                           remake=rem)
                del z, zh
            pre = new
        lin1, bn, _, drop, lin2 = self.mlp
        p1 = act_linears(pre[0], [lin1.weight], lin1.bias, bn=self.bn_layers[-1], relu=True,
                         dropout=self.dropout)[0]
        return act_linears(p1, [lin2.weight], lin2.bias, bn=bn, relu=True,
                           dropout=drop.p)[0]
