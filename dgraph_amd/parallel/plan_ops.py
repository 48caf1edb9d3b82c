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
