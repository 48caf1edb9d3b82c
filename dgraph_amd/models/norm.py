"""Synchronised batch normalisation over a vertex-partitioned graph (K-new-7).

Counterpart of ``DistributedBatchNorm1D`` (experiments/OGB-LSC/distributed_layers.py:77-214)
with its defects fixed:

* statistics are exact: every rank contributes ``(n_r, mean_r, M2_r)`` (one pass of the
  native ``bn_reduce`` kernel on GPU tensors — bf16 read as is, shifted fp32 partial sums,
  fp64 totals; ``torch.var_mean`` elsewhere) and the ranks' moments are combined with Chan's parallel
  formula after ONE all-gather of a ``[W, 2F+1]`` buffer — the reference divided the local
  *mean* by the global row count and all-reduced its numerator after using it;
* backward uses the textbook closed form
  ``dx = gamma * rstd * (dy - mean(dy) - x_hat * mean(dy * x_hat))`` whose two global
  means come from ONE all-reduce of a ``[2F]`` buffer (the reference issued four
  all-reduces, one of them with ``(var + eps) ** 2`` in place of ``** -1.5``);
* ``dgamma`` / ``dbeta`` are returned as rank-local partial sums: the replicated parameters'
  gradients are summed once by the data-parallel gradient sync (the reference all-reduced
  them inside the layer and again in DDP);
* the running variance uses the unbiased estimate (as ``torch.nn.BatchNorm1d``).

``recompute=True`` keeps only the input and recomputes ``x_hat`` in backward (the
reference's ``DistributedBN_with_Recompute``); otherwise ``x_hat`` is saved. The native
GPU path always recomputes (saving the bf16 input is cheaper than an fp32 ``x_hat``) and
can fuse the following ReLU (``forward(x, relu=True)``: the mask is recomputed from ``x``
in backward, nothing extra is stored).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn
from torch.autograd import Function


def _world(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _cdt(x: torch.Tensor) -> torch.dtype:
    return torch.float64 if x.dtype == torch.float64 else torch.float32


def _native_ok(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 2 and x.dtype in (torch.float32, torch.bfloat16)
            and (x.stride(1) == 1 or x.shape[1] <= 1))


def _ops():
    from .. import _native

    return _native.ops()


def _local_moments(x: torch.Tensor):
    """(n, mean, biased var) of this rank's rows, fp32 (fp64 for fp64 inputs)."""
    n, F = x.shape[0], x.shape[1]
    if n == 0:
        z = x.new_zeros(F, dtype=_cdt(x))
        return 0, z, z.clone()
    if _native_ok(x):
        # one pass over x (bf16 stays bf16): sums shifted by the first row, fp64 totals
        center = x[0].float().contiguous()
        s = _ops().bn_reduce(x, None, center, None, None, None, False, 0)
        m1 = s[0] / n
        mean = (center.double() + m1).float()
        var = (s[1] / n - m1 * m1).clamp_min(0).float()
        return n, mean, var
    var, mean = torch.var_mean(x.to(_cdt(x)), dim=0, unbiased=False)
    return n, mean, var


def global_moments(x: torch.Tensor, group=None):
    """(N, mean, biased var) of the rows of ``x`` over every rank of ``group`` (fp32)."""
    n, mean, var = _local_moments(x)
    F = x.shape[1]
    if _world(group) == 1:
        return float(n), mean, var
    packed = torch.cat([mean.new_tensor([float(n)]), mean, var * n])
    out = [torch.empty_like(packed) for _ in range(_world(group))]
    dist.all_gather(out, packed, group=group)
    allp = torch.stack(out)
    ns, means, m2s = allp[:, 0], allp[:, 1:F + 1], allp[:, F + 1:]
    N = float(ns.sum())
    gmean = (ns.unsqueeze(1) * means).sum(0) / max(N, 1.0)
    m2 = m2s.sum(0) + (ns.unsqueeze(1) * (means - gmean) ** 2).sum(0)
    return N, gmean, m2 / max(N, 1.0)


def _vec(p: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if p is None else p.reshape(-1).float().contiguous()


class BNState:
    """What the backward (and a recompute of the output) of one ``act(BN(x))`` needs: the
    global statistics, the affine parameters and the dropout seed — never the output."""

    __slots__ = ("mean", "rstd", "g", "b", "N", "relu", "p", "seed", "native", "group",
                 "gshape", "gdtype")


def bn_act_forward(x: torch.Tensor, gamma, beta, eps: float, group, relu: bool = False,
                   drop_p: float = 0.0):
    """``y = dropout(act(BN(x)))`` with global statistics -> ``(y, state, var)``.

    GPU (fp32/bf16 [N, F]): native kernels (csrc/kernels/batchnorm.hip) — one pass for the
    statistics and one fused normalise/affine/ReLU/dropout pass. The dropout keep mask is a
    function of (seed, element index) that :func:`bn_act_backward` and
    :func:`bn_act_recompute` regenerate."""
    st = BNState()
    N, mean, var = global_moments(x, group)
    st.seed = int(torch.randint(0, 1 << 62, (1,), dtype=torch.int64).item()) \
        if drop_p > 0 else 0
    st.p = float(drop_p)
    st.N, st.relu, st.group = N, relu, group
    st.mean, st.rstd = mean, torch.rsqrt(var + eps)
    st.gshape = None if gamma is None else gamma.shape
    st.gdtype = None if gamma is None else gamma.dtype
    st.g, st.b = _vec(gamma), _vec(beta)
    st.native = _native_ok(x)
    return bn_act_recompute(st, x), st, var


def bn_act_recompute(st: BNState, x: torch.Tensor) -> torch.Tensor:
    """The forward output again, bit for bit, from the saved input and state."""
    if st.native:
        return _ops().bn_apply(x, None, st.mean, st.rstd, st.g, st.b, None, None, st.relu, 0,
                               st.p, st.seed)
    y = (x.to(st.mean.dtype) - st.mean) * st.rstd
    if st.g is not None:
        y = y * st.g.to(st.mean.dtype) + st.b.to(st.mean.dtype)
    if st.relu:
        y = torch.relu(y)
    if st.p > 0:
        y = y * dropout_keep_mask(st.seed, *x.shape, x.device, st.p).to(y.dtype) / \
            (1.0 - st.p)
    return y.to(x.dtype)


def bn_act_backward(st: BNState, x: torch.Tensor, dy: torch.Tensor, xhat=None):
    """``(dx, dgamma, dbeta)`` of :func:`bn_act_forward` (``dgamma``/``dbeta`` rank-local;
    ``xhat``: the saved normalised input when the reference path did not recompute)."""
    mean, rstd, g, b = st.mean, st.rstd, st.g, st.b
    F = mean.numel()
    Nf = max(st.N, 1.0)
    p, seed = st.p, st.seed
    if st.native:
        dy = dy.to(x.dtype)
        if dy.stride(1) != 1 or dy.shape != x.shape:
            dy = dy.contiguous()
        s = _ops().bn_reduce(x, dy, mean, rstd, g, b, st.relu, 1, p, seed).float()
        sum_dy, sum_dy_xhat = s[0], s[1]
    else:
        if xhat is None:
            xhat = (x.to(mean.dtype) - mean) * rstd
        dyf = dy.to(mean.dtype)
        if p > 0:
            dyf = dyf * dropout_keep_mask(seed, *dyf.shape, dyf.device, p).to(dyf.dtype) / \
                (1.0 - p)
        if st.relu:
            pre = xhat * g.to(mean.dtype) + b.to(mean.dtype) if g is not None else xhat
            dyf = dyf * (pre > 0)
        sum_dy = dyf.sum(0)
        sum_dy_xhat = (dyf * xhat).sum(0)
    dgamma = dbeta = None
    if st.gshape is not None:
        dgamma = sum_dy_xhat.reshape(st.gshape).to(st.gdtype)
        dbeta = sum_dy.reshape(st.gshape).to(st.gdtype)
    glob = torch.cat([sum_dy, sum_dy_xhat])
    if _world(st.group) > 1:
        dist.all_reduce(glob, group=st.group)
    m_dy, m_dyx = glob[:F] / Nf, glob[F:] / Nf
    if st.native:
        dx = _ops().bn_apply(x, dy, mean, rstd, g, b, m_dy.contiguous(), m_dyx.contiguous(),
                             st.relu, 1, p, seed)
    else:
        dx = (dyf - m_dy - xhat * m_dyx) * rstd
        if g is not None:
            dx = dx * g.to(mean.dtype)
        dx = dx.to(dy.dtype)
    return dx, dgamma, dbeta


class _SyncBNFn(Function):
    """``y = act(BN(x))`` with global statistics; ``act`` is ReLU when ``relu``.

    GPU (fp32/bf16 [N, F]): native kernels (csrc/kernels/batchnorm.hip) — one pass for the
    statistics, one fused normalise/affine/ReLU pass, and in backward one fused reduction
    and one fused apply; only ``x`` is saved and nothing is materialised in fp32.
    Elsewhere: PyTorch reference math (``recompute`` saves ``x`` instead of ``x_hat``)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps: float, group, recompute: bool, box: list,
                relu: bool = False, drop_p: float = 0.0):
        y, st, var = bn_act_forward(x, gamma, beta, eps, group, relu, drop_p)
        box.append(st.N)
        ctx.st = st
        ctx.keep_xhat = not st.native and not recompute
        if ctx.keep_xhat:
            ctx.save_for_backward((x.to(st.mean.dtype) - st.mean) * st.rstd)
            ctx.xdtype = x.dtype
        else:
            ctx.save_for_backward(x)
        return y, st.mean, var

    @staticmethod
    def backward(ctx, dy, _dm, _dv):
        (saved,) = ctx.saved_tensors
        if ctx.keep_xhat:
            dx, dgamma, dbeta = bn_act_backward(ctx.st, saved, dy, xhat=saved)
        else:
            dx, dgamma, dbeta = bn_act_backward(ctx.st, saved, dy)
        return dx, dgamma, dbeta, None, None, None, None, None, None


def dropout_keep_mask(seed: int, N: int, F: int, device=None, p: float = 0.0) -> torch.Tensor:
    """The fused-dropout keep mask of the native BN kernels (csrc/kernels/batchnorm.hip
    ``dropout_keep``): keep (r, c) iff fmix32 of the element index r * F + c mixed with the
    64-bit seed is >= p * 2^32. A pure function of (seed, index): forward and backward (and
    the CPU reference and the GPU kernels) agree bit for bit."""
    M = 0xFFFFFFFF
    idx = torch.arange(N * F, dtype=torch.int64, device=device)
    lo, hi = idx & M, idx >> 32
    h = lo ^ (seed & M)
    h = h ^ ((((hi + (seed >> 32)) & M) * 0x9E3779B1) & M)
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & M
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & M
    h = h ^ (h >> 16)
    t = min(max(int(p * 4294967296.0), 1), 0xFFFFFFFF) if p > 0 else 0
    return (h >= t).view(N, F)


class DistributedBatchNorm1D(nn.Module):
    """Drop-in for the reference module (parameters ``gamma``/``beta`` of shape [1, F],
    buffers ``running_mean``/``running_var`` [1, F]); accepts [N, F] or [1, N, F] and
    returns the same rank it was given."""

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1,
                 affine: bool = True, track_running_stats: bool = True,
                 recompute: bool = False, group=None):
        super().__init__()
        if affine:
            self.gamma = nn.Parameter(torch.ones(1, num_features))
            self.beta = nn.Parameter(torch.zeros(1, num_features))
        else:
            self.register_parameter("gamma", None)
            self.register_parameter("beta", None)
        self.eps, self.momentum = eps, momentum
        self.track_running_stats = track_running_stats
        if track_running_stats:
            self.register_buffer("running_mean", torch.zeros(1, num_features))
            self.register_buffer("running_var", torch.ones(1, num_features))
            self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        else:
            self.running_mean = self.running_var = self.num_batches_tracked = None
        self.recompute = recompute
        self.group = group

    def _update_running(self, n: float, mean: torch.Tensor, var: torch.Tensor) -> None:
        if not self.track_running_stats:
            return
        with torch.no_grad():
            self.num_batches_tracked += 1
            unbiased = var * (n / max(n - 1.0, 1.0))
            self.running_mean.mul_(1 - self.momentum).add_(self.momentum * mean)
            self.running_var.mul_(1 - self.momentum).add_(self.momentum * unbiased)

    def forward(self, x: torch.Tensor, relu: bool = False, dropout: float = 0.0) -> torch.Tensor:
        """``BN(x)``, or ``relu(BN(x))`` fused into the same kernels when ``relu``; in
        training, ``dropout`` > 0 applies dropout after the activation in the same pass
        (mask regenerated in backward, never stored)."""
        squeeze = False
        if x.dim() == 3:
            if x.size(0) != 1:
                raise ValueError("only mini-batch size 1 is supported")
            x, squeeze = x[0], True
        elif x.dim() != 2:
            raise ValueError(f"Expected 2D or 3D input (got {x.dim()}D input)")
        if self.training or not self.track_running_stats:
            box: list = []
            y, mean, var = _SyncBNFn.apply(x, self.gamma, self.beta, self.eps, self.group,
                                           self.recompute, box, relu,
                                           float(dropout) if self.training else 0.0)
            if self.training:
                self._update_running(box[0], mean, var)
        else:
            y = (x.to(_cdt(x)) - self.running_mean) * torch.rsqrt(self.running_var + self.eps)
            if self.gamma is not None:
                y = y * self.gamma + self.beta
            if relu:
                y = torch.relu(y)
            y = y.to(x.dtype)
        return y.unsqueeze(0) if squeeze else y


def GetGlobalVal(local_val, group=None, device: Optional[torch.device] = None) -> float:
    """Sum of a scalar over all ranks (distributed_layers.py:210-214)."""
    dev = device or (torch.device("cuda", torch.cuda.current_device())
                     if torch.cuda.is_available() and dist.is_initialized()
                     and dist.get_backend(group) == "nccl" else torch.device("cpu"))
    t = torch.tensor([float(local_val)], device=dev)
    if _world(group) > 1:
        dist.all_reduce(t, group=group)
    return float(t.item())
