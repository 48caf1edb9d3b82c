"""Autograd-aware sparse primitives built on the native kernels.

* :func:`aggregate` — CSR SpMM (sum / mean / edge-weighted, multi-head); backward is the
  same kernel on the cached transposed CSR (or on the same CSR for symmetric patterns).
* :func:`gather` / :func:`scatter_sum` — vertex->edge gather and edge->vertex scatter-sum
  over a static :class:`~dgraph_amd.ops.csr.IndexMap`; each is the other's adjoint
  (the core contract of the reference, tests/test_NCCLCommPlan.py:100-111,297-307),
  and both are deterministic (segment sums, no float atomics).
* :func:`edge_softmax` — stable softmax over each destination's incoming edges.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch.autograd import Function

from . import kernels as K
from .csr import CSR, IndexMap


class _AggregateFn(Function):
    @staticmethod
    def forward(ctx, x, csr: CSR, edge_weight, mean: bool, heads: int):
        row_scale = csr.inv_degree() if mean else None
        out = K.spmm(csr.rowptr, csr.col, x, edge_weight=edge_weight,
                     row_scale=row_scale, heads=heads)
        ctx.csr, ctx.mean, ctx.heads = csr, mean, heads
        ctx.save_for_backward(x if edge_weight is not None and edge_weight.requires_grad else None,
                              edge_weight)
        return out

    @staticmethod
    def backward(ctx, g):
        csr: CSR = ctx.csr
        x_saved, ew = ctx.saved_tensors
        g = g.contiguous()
        gx = gw = None
        col_scale = csr.inv_degree() if ctx.mean else None
        if ctx.needs_input_grad[0]:
            if ew is None and csr.symmetric:
                gx = K.spmm(csr.rowptr, csr.col, g, col_scale=col_scale, heads=ctx.heads)
            else:
                t = csr.transpose()
                ew_t = None if ew is None else ew.reshape(csr.nnz, ctx.heads)[t.perm].contiguous()
                gx = K.spmm(t.rowptr, t.col, g, edge_weight=ew_t, col_scale=col_scale,
                            heads=ctx.heads)
        if ew is not None and ctx.needs_input_grad[2]:
            # d w[j,h] = row_scale[r] * <g[r, h-slice], x[c_j, h-slice]>  (SDDMM)
            rows = csr.row_ids()
            H = ctx.heads
            cdt = torch.float64 if ew.dtype == torch.float64 else torch.float32
            gr = g.to(cdt)[rows].view(csr.nnz, H, -1)
            xc = x_saved.to(cdt)[csr.col.long()].view(csr.nnz, H, -1)
            gw = (gr * xc).sum(-1)
            if ctx.mean:
                gw = gw * csr.inv_degree()[rows].unsqueeze(1)
            gw = gw.reshape(ew.shape).to(ew.dtype)
        return gx, None, gw, None, None


def aggregate(
    x: torch.Tensor,
    csr: CSR,
    edge_weight: Optional[torch.Tensor] = None,
    reduce: str = "sum",
    heads: int = 1,
) -> torch.Tensor:
    """``out[r] = reduce_{j in N(r)} w_j * x[j]`` over the CSR rows.

    ``edge_weight`` is ``[nnz]`` or ``[nnz, heads]`` in CSR slot order; with heads > 1
    the feature dim is split into ``heads`` equal slices, each scaled by its head weight.
    """
    if reduce not in ("sum", "mean"):
        raise ValueError(f"unsupported reduce {reduce!r}")
    ew = None
    if edge_weight is not None:
        ew = edge_weight.reshape(csr.nnz, heads)  # native path casts to fp32 itself
        if ew.dtype not in (torch.float32, torch.float64):
            ew = ew.float()
    return _AggregateFn.apply(x.contiguous(), csr, ew, reduce == "mean", heads)


class _GatherFn(Function):
    @staticmethod
    def forward(ctx, x, imap: IndexMap):
        ctx.imap = imap
        ctx.n = x.shape[0]
        return K.gather_rows(x, imap.idx)

    @staticmethod
    def backward(ctx, g):
        t = ctx.imap.transpose_csr()
        gx = K.spmm(t.rowptr, t.col, g.contiguous(), split=ctx.imap.transpose_split())
        return gx, None


class _ScatterSumFn(Function):
    @staticmethod
    def forward(ctx, x, imap: IndexMap):
        ctx.imap = imap
        t = imap.transpose_csr()
        return K.spmm(t.rowptr, t.col, x.contiguous(), split=imap.transpose_split())

    @staticmethod
    def backward(ctx, g):
        return K.gather_rows(g.contiguous(), ctx.imap.idx), None


def gather(x: torch.Tensor, imap: IndexMap) -> torch.Tensor:
    """``y[i] = x[idx[i]]``; backward is the deterministic scatter-sum."""
    return _GatherFn.apply(x, imap)


def scatter_sum(x: torch.Tensor, imap: IndexMap) -> torch.Tensor:
    """``y[v] = sum_{i: idx[i]=v} x[i]`` (``imap.num_src`` output rows)."""
    return _ScatterSumFn.apply(x, imap)


class _EdgeSoftmaxFn(Function):
    @staticmethod
    def forward(ctx, scores, rowptr):
        alpha = K.edge_softmax_fwd(rowptr, scores)
        ctx.save_for_backward(rowptr, alpha)
        return alpha

    @staticmethod
    def backward(ctx, g):
        rowptr, alpha = ctx.saved_tensors
        return K.edge_softmax_bwd(rowptr, alpha, g), None


def edge_softmax(scores: torch.Tensor, csr: CSR) -> torch.Tensor:
    """Softmax of ``scores[nnz(, H)]`` (CSR slot order) over each row's edges."""
    return _EdgeSoftmaxFn.apply(scores, csr.rowptr)
