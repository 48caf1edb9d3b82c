"""Row LayerNorm with an optional fused residual add (csrc/kernels/layernorm.hip).

``layer_norm(x, weight, bias, eps, residual)`` = ``F.layer_norm(x, ...) + residual``;
GPU tensors run the native kernel (fp32 statistics, fp32 dgamma/dbeta partial sums per
block), CPU tensors use PyTorch (the numerics reference).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F
from torch.autograd import Function

from .. import _native


class _LayerNormFn(Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, eps: float):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        w = None if weight is None else weight.float().contiguous()
        b = None if bias is None else bias.float().contiguous()
        r = None if residual is None else residual.reshape(x2.shape).to(x2.dtype).contiguous()
        y, mean, rstd = _native.ops().layer_norm_fwd(x2, w, b, r, float(eps))
        ctx.save_for_backward(x2, mean, rstd, w if w is not None else mean)
        ctx.has_w = weight is not None
        ctx.wdt = None if weight is None else weight.dtype
        ctx.shape = shape
        ctx.has_res = residual is not None
        return y.reshape(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, mean, rstd, w = ctx.saved_tensors
        dy2 = dy.reshape(x2.shape).to(x2.dtype).contiguous()
        dx, dg, db = _native.ops().layer_norm_bwd(dy2, x2, mean, rstd,
                                                  w if ctx.has_w else None)
        dw = dg.to(ctx.wdt) if ctx.has_w and ctx.needs_input_grad[1] else None
        dbias = db.to(ctx.wdt) if ctx.has_w and ctx.needs_input_grad[2] else None
        dres = dy if ctx.has_res and ctx.needs_input_grad[3] else None
        return dx.reshape(ctx.shape), dw, dbias, dres, None


def layer_norm(x: torch.Tensor, weight: Optional[torch.Tensor], bias: Optional[torch.Tensor],
               eps: float = 1e-5, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16):
        return _LayerNormFn.apply(x, weight, bias, residual, eps)
    y = F.layer_norm(x, (x.shape[-1],), weight, bias, eps)
    return y if residual is None else y + residual
