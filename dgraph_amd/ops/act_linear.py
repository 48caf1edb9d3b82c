"""``outs_i = act(x) W_i^T (+ b)`` with ``act`` = dropout(ReLU(BatchNorm(x))) recomputed in
backward instead of stored (the fp32 R-GCN's memory-lean layer, ``models/rgcn.py``).

A BN'd activation feeds exactly the GEMMs of the next layer (skip and relation transforms
of one source type, or an MLP linear); only the pre-BN input is saved, the normalised
activation is rebuilt for the weight gradients (one elementwise pass) — at MAG240M scale
that drops one [rows, hidden] fp32 tensor per (layer, node type) from the saved set (15.6 GB
each on one GPU's 1/8 share). The reference keeps both (experiments/OGB-LSC/RGAT.py:320-349
runs BN, ReLU, dropout and the next layer's linears as separate autograd nodes;
distributed_layers.py:77-214 saves ``x_hat`` unless recomputing).

GPU fp32: the GEMMs run on the exact-f32 MFMA kernel (``ops.f32.gemm_f32``, bias fused),
``dy = sum_i g_i W_i`` two terms per call with the running sum chained through ``cin``,
and ``dW_i`` on the split-M MFMA weight-gradient accumulator (``ops.f32.WgradAcc``); widths
the kernels do not tile (e.g. 153 classes) fall back to the library GEMM. Elsewhere
(CPU, bf16): plain PyTorch math, the numerics oracle.
"""
from __future__ import annotations

from typing import List, Sequence

import torch
from torch.autograd import Function

from . import f32 as F32
from . import kernels as K


def _wgrad(g: torch.Tensor, y: torch.Tensor, W: torch.Tensor, bias: bool = False):
    """``g^T y`` in W's layout [N, K] (``bias``: and ``g``'s column sums, from the same
    kernel pass on the GPU)."""
    r = F32.linear_wgrad(g, y, W, bias=bias)
    if r is not None:
        return r
    adt = torch.float64 if g.dtype == torch.float64 else torch.float32
    dW = (g.t().to(adt) @ y.to(adt)).to(W.dtype)
    if not bias:
        return dW
    return dW, (K.col_sum(g) if g.is_cuda else g.sum(0))


def _tiled(y: torch.Tensor, W: torch.Tensor) -> bool:
    """Does ``F32.linear_fwd(y, W)`` run on the MFMA kernel (else the library GEMM)?"""
    N, K = W.shape
    return F32._on(y) and K % 32 == 0 and F32.tileable(N)


class _ActLinearsFn(Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, bias, bn, relu: bool, drop_p: float, *Ws):
        st = None
        if bn is not None:
            from ..models.norm import bn_act_forward

            y, st, var = bn_act_forward(x, gamma, beta, bn.eps, bn.group, relu, drop_p)
            bn._update_running(st.N, st.mean, var)
        else:
            y = x
        # narrow outputs (widths the MFMA kernels do not tile, e.g. RGAT's per-head
        # destination scores) as ONE library GEMM over their stacked weights: the input is
        # read once for all of them, not once each
        narrow = [i for i, W in enumerate(Ws) if (i > 0 or bias is None) and
                  not _tiled(y, W)]
        outs = [None] * len(Ws)
        if len(narrow) > 1:
            Wn = torch.cat([Ws[i] for i in narrow]).to(y.dtype)
            zn = y @ Wn.t()
            o = 0
            for i in narrow:
                n = Ws[i].shape[0]
                outs[i] = zn[:, o:o + n]
                o += n
        for i, W in enumerate(Ws):
            if outs[i] is None:
                outs[i] = F32.linear_fwd(y, W, bias if i == 0 else None)
        del y
        ctx.st = st
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, *Ws)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        x, *Ws = ctx.saved_tensors
        st = ctx.st
        if st is not None:
            from ..models.norm import bn_act_recompute

            y = bn_act_recompute(st, x)
        else:
            y = x
        live = any(g is not None for g in gs)
        gs_c = [None if g is None else (g if g.stride(1) == 1 and g.is_contiguous()
                                        else g.contiguous()) for g in gs]
        dWs = []
        db = None
        want_b = ctx.has_bias and ctx.needs_input_grad[3] and gs_c[0] is not None
        # narrow weight gradients (no MFMA tiling) as ONE library GEMM over their stacked
        # output gradients: the activation is read once for all of them
        narrow = [i for i, (g, W) in enumerate(zip(gs_c, Ws)) if g is not None and
                  not (i == 0 and want_b) and not F32.wgrad_tiled(g, y, W)]
        done = {}
        if len(narrow) > 1:
            gn = torch.cat([gs_c[i] for i in narrow], 1)
            adt = torch.float64 if gn.dtype == torch.float64 else torch.float32
            dWn = gn.t().to(adt) @ y.to(adt)
            o = 0
            for i in narrow:
                n = Ws[i].shape[0]
                done[i] = dWn[o:o + n].to(Ws[i].dtype)
                o += n
        for i, (g, W) in enumerate(zip(gs_c, Ws)):
            if i in done:
                dWs.append(done[i])
            elif g is None:
                dWs.append(None)
            elif i == 0 and want_b:
                dW, db = _wgrad(g, y, W, bias=True)
                dWs.append(dW)
                db = db.to(Ws[0].dtype)
            else:
                dWs.append(_wgrad(g, y, W))
        dx = dgamma = dbeta = None
        need_x = ctx.needs_input_grad[0] or (st is not None and (ctx.needs_input_grad[1]
                                                                 or ctx.needs_input_grad[2]))
        if need_x and live:
            dy = F32.linear_dgrad([g for g, W in zip(gs_c, Ws) if g is not None],
                     [W for g, W in zip(gs_c, Ws) if g is not None])
            if st is not None:
                from ..models.norm import bn_act_backward

                del y
                dx, dgamma, dbeta = bn_act_backward(st, x, dy)
            else:
                dx = dy
        return (dx, dgamma, dbeta, db, None, None, None, *dWs)


def act_linears(x: torch.Tensor, Ws: Sequence[torch.Tensor], bias=None, bn=None,
                relu: bool = False, dropout: float = 0.0) -> List[torch.Tensor]:
    """``[act(x) W_i^T (+ bias on the first)]`` with ``act`` = dropout(relu?(bn(x))) when
    ``bn`` (a :class:`~dgraph_amd.models.norm.DistributedBatchNorm1D` in training mode) is
    given, identity otherwise. Saves ``x`` only."""
    if bn is not None and not bn.training:
        x = bn(x, relu=relu)
        bn = None
    elif bn is None and (relu or dropout):
        raise ValueError("act_linears: relu/dropout need a BatchNorm")
    gamma = beta = None
    if bn is not None:
        gamma, beta = bn.gamma, bn.beta
    return list(_ActLinearsFn.apply(x, gamma, beta, bias, bn, bool(relu),
                                    float(dropout) if bn is not None else 0.0, *Ws))
