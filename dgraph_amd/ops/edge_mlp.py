"""Autograd ops for edge MLPs whose first layer acts on a concatenation
``[x_src || x_dst (|| e)]`` (GCN.py:43-65, GraphCast layers.py:146-216, RGAT.py:147-153).

The first Linear distributes over the concatenation, ``W [a || b || e] + bias =
(a W_a^T + bias) + b W_b^T + e W_e^T``, so the per-edge GEMM over ``E x (2F + F_e)``
becomes vertex-level GEMMs (MFMA via hipBLASLt) and gather-bound fused kernels
(csrc/kernels/edge_fused.hip):

* :func:`pair_relu_aggregate` — ``out[i] = sum_{j in N(i)} relu(P[i] + Q[j])`` with no
  per-edge intermediate at all (forward and both backward terms are CSR kernels);
* :func:`edge_pre_activation` — ``h[e] = act(Y[e] + P[src[e]] + Q[dst[e]])`` for deeper edge
  MLPs (the pre-activation is recomputed in backward, never stored).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch.autograd import Function

from . import kernels as K
from .csr import CSR, IndexMap


class _PairReluAggFn(Function):
    @staticmethod
    def forward(ctx, P, Q, csr: CSR):
        P = P.contiguous()
        Q = Q.contiguous()
        out = K.pair_relu(csr.rowptr, csr.col, 0, P, Q)
        ctx.csr = csr
        ctx.save_for_backward(P, Q)
        return out

    @staticmethod
    def backward(ctx, g):
        P, Q = ctx.saved_tensors
        csr: CSR = ctx.csr
        g = g.contiguous().to(P.dtype)
        dP = dQ = None
        if ctx.needs_input_grad[0]:
            dP = K.pair_relu(csr.rowptr, csr.col, 1, P, Q, rowmul=g)
        if ctx.needs_input_grad[1]:
            t = csr.transpose()
            dQ = K.pair_relu(t.rowptr, t.col, 2, Q, P, gat2=g)
            if dQ.shape[0] < Q.shape[0]:  # pragma: no cover - transpose covers all columns
                dQ = torch.cat([dQ, dQ.new_zeros(Q.shape[0] - dQ.shape[0], dQ.shape[1])])
        return dP, dQ, None


def pair_relu_aggregate(P: torch.Tensor, Q: torch.Tensor, csr: CSR) -> torch.Tensor:
    """``out[i] = sum_{j in N(i)} relu(P[i] + Q[j])`` over ``csr`` (rows i, columns j)."""
    if P.shape[0] < csr.num_rows or Q.shape[0] < csr.num_cols:
        raise ValueError("P/Q have fewer rows than the CSR's rows/columns")
    if P.dtype != Q.dtype:
        Q = Q.to(P.dtype)
    return _PairReluAggFn.apply(P, Q, csr)


class _EdgePreActFn(Function):
    @staticmethod
    def forward(ctx, Y, P, Q, src_map: Optional[IndexMap], dst_map: Optional[IndexMap],
                act: str):
        ref = next(t for t in (Y, P, Q) if t is not None)
        E = Y.shape[0] if Y is not None else (src_map.idx.numel() if src_map is not None
                                              else dst_map.idx.numel())
        Fdim = ref.shape[1]
        src = src_map.idx.long() if (P is not None) else None
        dst = dst_map.idx.long() if (Q is not None) else None
        args = dict(Y=None if Y is None else Y.contiguous(),
                    P=None if P is None else P.contiguous(), src=src,
                    Q=None if Q is None else Q.contiguous(), dst=dst)
        out = K.gather_add_act(E, Fdim, act=act, dtype=ref.dtype, device=ref.device, **args)
        ctx.args, ctx.act, ctx.E, ctx.F = args, act, E, Fdim
        ctx.src_map, ctx.dst_map = src_map, dst_map
        ctx.save_for_backward(*(t for t in (args["Y"], args["P"], args["Q"]) if t is not None))
        return out

    @staticmethod
    def backward(ctx, g):
        a = ctx.args
        d = K.gather_add_act(ctx.E, ctx.F, gin=g.contiguous().to(
            next(t for t in (a["Y"], a["P"], a["Q"]) if t is not None).dtype),
            act=ctx.act, **a)
        dY = d if (a["Y"] is not None and ctx.needs_input_grad[0]) else None
        dP = dQ = None
        if a["P"] is not None and ctx.needs_input_grad[1]:
            t = ctx.src_map.transpose_csr()
            dP = K.spmm(t.rowptr, t.col, d, split=ctx.src_map.transpose_split())
        if a["Q"] is not None and ctx.needs_input_grad[2]:
            t = ctx.dst_map.transpose_csr()
            dQ = K.spmm(t.rowptr, t.col, d, split=ctx.dst_map.transpose_split())
        return dY, dP, dQ, None, None, None


def edge_pre_activation(Y: Optional[torch.Tensor], P: Optional[torch.Tensor],
                        Q: Optional[torch.Tensor], src_map: Optional[IndexMap] = None,
                        dst_map: Optional[IndexMap] = None, act: str = "none") -> torch.Tensor:
    """``h[e] = act(Y[e] + P[src[e]] + Q[dst[e]])``; ``src_map``/``dst_map`` are
    :class:`IndexMap` s over the vertex rows of ``P``/``Q`` (their transposed CSRs make the
    backward scatter-sums deterministic)."""
    dts = {t.dtype for t in (Y, P, Q) if t is not None}
    if len(dts) > 1:
        dt = next(t for t in (Y, P, Q) if t is not None).dtype
        Y = None if Y is None else Y.to(dt)
        P = None if P is None else P.to(dt)
        Q = None if Q is None else Q.to(dt)
    return _EdgePreActFn.apply(Y, P, Q, src_map, dst_map, act)
