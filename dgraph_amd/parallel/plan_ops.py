"""Plan-based distributed gather / scatter-sum autograd ops (API generation G2).

Semantics of the reference's ``CommPlan_GatherFunction`` / ``CommPlan_ScatterFunction``
(DGraph/distributed/nccl/_torch_func_impl.py:27-352), executed on a
:class:`~dgraph_amd.plan.nccl_plan.CompiledPlan`:

gather  ``Y[e] = X_global[g(e)]``
    fwd: local rows by ``copy_rows``; boundary rows packed by the plan's vertex index,
         one all-to-all-v, unpacked by the buffer map.
    bwd: edge grads pre-aggregated per (peer, vertex) with a segment sum (I4), reverse
         all-to-all-v, then segment-summed into the owner rows — no float atomics.
scatter ``Y[v] = sum_{e: g(e)=v} X[e]`` — the adjoint of gather (and vice versa).

Outputs keep the input dtype (bf16 stays bf16; the reference forced fp32,
_torch_func_impl.py:57-59). Inputs are ``[1, N, F]`` (batch 1, as the reference asserts)
or ``[N, F]``.
"""
from __future__ import annotations

import torch
from torch.autograd import Function

from ..ops import kernels as K
from ..plan.nccl_plan import CompiledPlan, NCCLGraphCommPlan


def _gather_fwd(cp: CompiledPlan, x: torch.Tensor) -> torch.Tensor:
    p = cp.plan
    F = x.shape[1]
    y = torch.zeros(p.num_local_edges, F, dtype=x.dtype, device=x.device)
    if p.local_edge_idx.numel():
        K.copy_rows(x, src_idx=p.local_vertex_idx, dst_idx=p.local_edge_idx, out=y)
    send = K.gather_rows(x, p.boundary_vertex_idx) if p.boundary_vertex_idx.numel() else \
        x.new_zeros(0, F)
    recv = cp.a2a_v2e(send)
    if p.boundary_edge_idx.numel():
        K.copy_rows(recv, src_idx=p.boundary_edge_buffer_map, dst_idx=p.boundary_edge_idx, out=y)
    return y


def _scatter_fwd(cp: CompiledPlan, x: torch.Tensor) -> torch.Tensor:
    p = cp.plan
    F = x.shape[1]
    # pre-aggregate boundary contributions per (peer, vertex) and ship them first so the
    # local segment sum overlaps the exchange
    buf = K.spmm(cp.pack.rowptr, cp.pack.col, x) if cp.pack.num_rows else x.new_zeros(0, F)
    recv, work = cp.a2a_e2v(buf, async_op=True)
    y = K.spmm(cp.local.rowptr, cp.local.col, x)
    work.wait()
    if cp.unpack.nnz:
        K.spmm(cp.unpack.rowptr, cp.unpack.col, recv, out=y, beta=1.0)
    return y


class CommPlan_GatherFunction(Function):
    @staticmethod
    def forward(ctx, x, plan: NCCLGraphCommPlan, group=None):
        ctx.cp = plan.compiled(group)
        return _gather_fwd(ctx.cp, x.contiguous())

    @staticmethod
    def backward(ctx, g):
        return _scatter_fwd(ctx.cp, g.contiguous()), None, None


class CommPlan_ScatterFunction(Function):
    @staticmethod
    def forward(ctx, x, plan: NCCLGraphCommPlan, group=None):
        ctx.cp = plan.compiled(group)
        return _scatter_fwd(ctx.cp, x.contiguous())

    @staticmethod
    def backward(ctx, g):
        return _gather_fwd(ctx.cp, g.contiguous()), None, None


def _squeeze_batch(x: torch.Tensor):
    if x.dim() == 3:
        if x.shape[0] != 1:
            raise ValueError("batch dimension must be 1")
        return x[0], True
    if x.dim() == 1:
        return x.unsqueeze(1), False
    return x, False


def plan_gather(x: torch.Tensor, plan: NCCLGraphCommPlan, group=None) -> torch.Tensor:
    x2, batched = _squeeze_batch(x)
    y = CommPlan_GatherFunction.apply(x2, plan, group)
    return y.unsqueeze(0) if batched else y


def plan_scatter(x: torch.Tensor, plan: NCCLGraphCommPlan, group=None) -> torch.Tensor:
    x2, batched = _squeeze_batch(x)
    y = CommPlan_ScatterFunction.apply(x2, plan, group)
    return y.unsqueeze(0) if batched else y


# ----------------------------------------------------------------------- grouped gather
class _Grouped:
    """Several plans' vertex->edge exchanges as ONE all-to-all-v: per peer, the plans'
    segments back to back (plan order). ``send_pos[t]`` / ``recv_pos[t]``: where plan t's
    send / receive rows sit in the combined buffers."""

    def __init__(self, cps, group):
        from ..comm.alltoallv import AllToAllV

        W = len(cps[0].a2a_v2e.send_splits)
        dev = cps[0].plan.boundary_vertex_idx.device
        ss = [list(cp.a2a_v2e.send_splits) for cp in cps]
        rs = [list(cp.a2a_v2e.recv_splits) for cp in cps]
        tot_s = [sum(s[p] for s in ss) for p in range(W)]
        tot_r = [sum(r[p] for r in rs) for p in range(W)]
        self.a2a = AllToAllV(tot_s, tot_r, group)

        def positions(splits, tot):
            out = []
            base = [0] * W
            for p in range(1, W):
                base[p] = base[p - 1] + tot[p - 1]
            done = [0] * W  # rows of earlier plans in peer p's segment
            for sp in splits:
                idx = []
                for p in range(W):
                    idx.append(torch.arange(sp[p], dtype=torch.long) + base[p] + done[p])
                    done[p] += sp[p]
                out.append(torch.cat(idx).to(dev) if idx else
                           torch.zeros(0, dtype=torch.long, device=dev))
            return out

        self.send_pos = positions(ss, tot_s)
        self.recv_pos = positions(rs, tot_r)
        self.n_send, self.n_recv = sum(tot_s), sum(tot_r)


_GROUPED: dict = {}


def _grouped(cps, group) -> _Grouped:
    key = (tuple(id(cp) for cp in cps), id(group))
    g = _GROUPED.get(key)
    if g is None or any(a is not b for a, b in zip(g.cps, cps)):
        g = _Grouped(cps, group)
        g.cps = tuple(cps)
        _GROUPED[key] = g
    return g


def _grouped_gather_fwd(cps, gp: _Grouped, xs):
    F = xs[0].shape[1]
    send = xs[0].new_empty(gp.n_send, F)
    for cp, x, pos in zip(cps, xs, gp.send_pos):
        if pos.numel():
            K.copy_rows(x, src_idx=cp.plan.boundary_vertex_idx, dst_idx=pos, out=send)
    recv = gp.a2a(send)
    ys = []
    for cp, x, pos in zip(cps, xs, gp.recv_pos):
        p = cp.plan
        y = torch.zeros(p.num_local_edges, F, dtype=x.dtype, device=x.device)
        if p.local_edge_idx.numel():
            K.copy_rows(x, src_idx=p.local_vertex_idx, dst_idx=p.local_edge_idx, out=y)
        if p.boundary_edge_idx.numel():
            mine = K.gather_rows(recv, pos)
            K.copy_rows(mine, src_idx=p.boundary_edge_buffer_map, dst_idx=p.boundary_edge_idx,
                        out=y)
        ys.append(y)
    return ys


def _grouped_scatter_fwd(cps, gp: _Grouped, gs):
    """Adjoint of :func:`_grouped_gather_fwd`: one reverse all-to-all-v for every plan."""
    F = gs[0].shape[1]
    back = gs[0].new_empty(gp.n_recv, F)
    for cp, g, pos in zip(cps, gs, gp.recv_pos):
        if pos.numel():
            buf = K.spmm(cp.pack.rowptr, cp.pack.col, g) if cp.pack.num_rows else \
                g.new_zeros(0, F)
            K.copy_rows(buf, dst_idx=pos, out=back)
    recv, work = gp.a2a.reversed()(back, async_op=True)
    outs = [K.spmm(cp.local.rowptr, cp.local.col, g) for cp, g in zip(cps, gs)]
    work.wait()
    for cp, o, pos in zip(cps, outs, gp.send_pos):
        if cp.unpack.nnz:
            K.spmm(cp.unpack.rowptr, cp.unpack.col, K.gather_rows(recv, pos), out=o, beta=1.0)
    return outs


class _GroupedGatherFn(Function):
    @staticmethod
    def forward(ctx, plans, group, *xs):
        cps = [p.compiled(group) for p in plans]
        gp = _grouped(cps, group)
        ctx.cps, ctx.gp = cps, gp
        return tuple(_grouped_gather_fwd(cps, gp, [x.contiguous() for x in xs]))

    @staticmethod
    def backward(ctx, *gs):
        gs = [g.contiguous() for g in gs]
        return (None, None, *_grouped_scatter_fwd(ctx.cps, ctx.gp, gs))


def plan_gather_grouped(xs, plans, group=None):
    """``[plan_gather(x_t, plan_t)]`` for every t with ONE all-to-all-v forward and ONE in
    backward (the reference issues one per call, RGAT.py:171-201). Inputs ``[N_t, F]`` of
    one width."""
    if len({x.shape[1] for x in xs}) != 1:
        raise ValueError("plan_gather_grouped: inputs must share their width")
    return list(_GroupedGatherFn.apply(tuple(plans), group, *xs))
