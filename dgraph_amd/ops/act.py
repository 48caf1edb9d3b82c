"""Linear layer(s) + bias + pointwise activation as one autograd node.

``linear_act([(x_1, W_1), (x_2, W_2), ...], b, "silu")`` = ``act(sum_i x_i W_i^T + b)``:
the MeshGraphMLP hidden layers of GraphCast (Linear -> SiLU, experiments/GraphCast/
layers.py:24-75; the node block's first Linear over ``[x || agg]`` is two terms, so no
concatenation and no separate add). GPU:
  forward  — the bias-free product (native MFMA dual GEMM, two terms per launch — bf16, or
             exact-f32 at fp32 — or the library GEMM for untiled widths) then ONE fused
             bias + activation pass (csrc/kernels/act.hip);
  backward — ONE pass computes ``dz = dy * act'(z + b)`` and the bias gradient's column
             sums together; ``dx_i = dz W_i``, ``dW_i`` by the split-K weight gradient.
PyTorch's path is addmm + silu forward and silu_backward + a column reduction (an extra
read of dz) backward. CPU tensors run the same math in PyTorch (the tests' reference).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as Fn

from .. import _native
from . import f32 as F32
from .dense import (_DEFER, _auto_rows_per_chunk, _native_linear_sum_ok, _wgrad_chunk,
                    defer_param_grads, dual_gemm, dual_gemm_shape_ok,
                    wgrad)

ACTS = {"identity": 0, "silu": 1, "relu": 2}


def _act_ref(z: torch.Tensor, act: int) -> torch.Tensor:
    if act == 1:
        return Fn.silu(z)
    if act == 2:
        return torch.relu(z)
    return z


def _f32_mm_ok(xs, Ws) -> bool:
    return (F32.LINEAR_ON and xs[0].is_cuda and xs[0].shape[0] > 0
            and all(x.dtype == torch.float32 and x.dim() == 2 and x.stride(1) == 1
                    and x.shape[1] % 32 == 0 for x in xs)
            and F32.tileable(Ws[0].shape[0]))


def _native_ok(z: torch.Tensor) -> bool:
    """Shapes csrc/kernels/act.hip takes: a row of F elements is covered by at most 256
    threads — vectors of 8 (bf16) / 4 (fp32) when F and the row stride allow, else one
    element per thread (F <= 256)."""
    if not (z.is_cuda and z.dtype in (torch.float32, torch.bfloat16) and z.dim() == 2):
        return False
    F = z.shape[1]
    vec = 8 if z.dtype == torch.bfloat16 else 4
    if F % vec == 0 and z.stride(0) % vec == 0:
        return F // vec <= 256
    return F <= 256


class _LinearActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, b, act: int, *flat):
        xs, Ws = list(flat[0::2]), list(flat[1::2])
        native_mm = _native_linear_sum_ok(xs, Ws, None)
        if native_mm:
            z = torch.empty(xs[0].shape[0], Ws[0].shape[0], dtype=xs[0].dtype,
                            device=xs[0].device)
            cin = None
            for k in range(0, len(xs), 2):
                two = k + 1 < len(xs)
                dual_gemm(xs[k], Ws[k].to(xs[k].dtype), xs[k + 1] if two else None,
                          Ws[k + 1].to(xs[k].dtype) if two else None, cin=cin, out=z)
                cin = z
        elif _f32_mm_ok(xs, Ws):
            # fp32: the exact-f32 MFMA GEMM, two terms per launch, running sum through cin
            z = None
            for k in range(0, len(xs), 2):
                two = k + 1 < len(xs)
                z = F32.gemm_f32(xs[k], Ws[k].t().contiguous(), xs[k + 1] if two else None,
                                 Ws[k + 1].t().contiguous() if two else None, cin=z, out=z)
        else:
            z = Fn.linear(xs[0], Ws[0])
            for x, W in zip(xs[1:], Ws[1:]):
                z = z + Fn.linear(x, W)
        bf = None if b is None else b.float().contiguous()
        if _native_ok(z):
            y = torch.empty_like(z)
            _native.ops().bias_act(z, bf, int(act), y)
        else:
            y = _act_ref(z if b is None else z + b.to(z.dtype), act)
        ctx.save_for_backward(z, bf if bf is not None else z.new_empty(0), *flat)
        ctx.act, ctx.has_b, ctx.native_mm = act, b is not None, native_mm
        ctx.bdt = None if b is None else b.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        z, bf, *flat = ctx.saved_tensors
        xs, Ws = flat[0::2], flat[1::2]
        bf = bf if ctx.has_b else None
        dy = dy.contiguous()
        if dy.is_cuda and dy.data_ptr() % 16:
            dy = dy.clone()  # the vector lanes need 16-B aligned rows
        if _native_ok(z):
            dz = torch.empty_like(z)
            db = _native.ops().bias_act_bwd(dy, z, bf, int(ctx.act), dz)
        else:
            zz = (z if bf is None else z + bf.to(z.dtype)).detach().requires_grad_(True)
            with torch.enable_grad():
                yy = _act_ref(zz, ctx.act)
            (dz,) = torch.autograd.grad(yy, zz, dy)
            db = dz.to(torch.float64 if dz.dtype == torch.float64 else torch.float32).sum(0)
        grads: List[Optional[torch.Tensor]] = []
        wi = [i for i in range(len(Ws)) if ctx.needs_input_grad[3 + 2 * i]]
        deferred = dz.is_cuda and _DEFER.active and bool(wi)
        for i, (x, W) in enumerate(zip(xs, Ws)):
            dx = dW = None
            if ctx.needs_input_grad[2 + 2 * i]:
                if ctx.native_mm and dual_gemm_shape_ok(x.shape[1], W.shape[0]):
                    dx = dual_gemm(dz, W.to(dz.dtype).t().contiguous())
                else:
                    dx = F32.linear_dgrad([dz], [W])
            if ctx.needs_input_grad[3 + 2 * i] and not deferred:
                dW = F32.linear_wgrad(dz, x, W)  # fp32: split-M MFMA accumulator
                if dW is None and dz.is_cuda:
                    L = dz.shape[0]
                    dW = wgrad(dz, x.contiguous(),
                               0 if L >= 1 << 23 else _auto_rows_per_chunk(L))
                elif dW is None:
                    adt = torch.float64 if dz.dtype == torch.float64 else torch.float32
                    dW = dz.t().to(adt) @ x.to(adt)
                dW = dW.to(W.dtype)
            grads += [dx, dW]
        if deferred:
            def comp():
                out = []
                for i in wi:
                    r = F32.linear_wgrad(dz, xs[i], Ws[i])
                    out.append(r if r is not None else
                               wgrad(dz, xs[i].contiguous(), _wgrad_chunk(dz.shape[0])))
                return out

            if not defer_param_grads([Ws[i] for i in wi], comp,
                                     keep_alive=(dz, *[xs[i] for i in wi])):
                for i, r in zip(wi, comp()):  # not deferrable: the normal path
                    grads[2 * i + 1] = r.to(Ws[i].dtype)
        dbo = db.to(ctx.bdt) if ctx.has_b and ctx.needs_input_grad[0] else None
        return (dbo, None, *grads)


def linear_act(terms: Sequence[Tuple[torch.Tensor, torch.Tensor]], b: Optional[torch.Tensor],
               act: str = "silu") -> torch.Tensor:
    """``act(sum_i x_i W_i^T + b)`` for ``terms = [(x_i, W_i), ...]`` (2-D ``x_i``)."""
    xs = [x for x, _ in terms]
    Ws = [W for _, W in terms]
    if torch.is_autocast_enabled() and xs[0].is_cuda:
        dt = torch.get_autocast_dtype("cuda")
        xs = [x.to(dt) for x in xs]
        Ws = [W.to(dt) for W in Ws]
    else:
        Ws = [W.to(xs[0].dtype) if W.dtype != xs[0].dtype else W for W in Ws]
    shape = xs[0].shape
    xs = [x.reshape(-1, x.shape[-1]) for x in xs]
    flat = [t for pair in zip(xs, Ws) for t in pair]
    y = _LinearActFn.apply(b, ACTS[act], *flat)
    return y.reshape(*shape[:-1], y.shape[-1])
