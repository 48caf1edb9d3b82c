"""Fused fp32 relation attention with its exact adjoint (the lean RGAT layer).

For one relation (destination rows i, source columns j over ``[local sources | halo rows]``)
and per head k (channels ``[kD, (k+1)D)`` of ``C = heads * D``)::

    ss_j  = z_j[head k] . a_src[k]                        (source score, from z)
    e_ij  = leaky_relu(sd_i + ss_j, 0.2)                  (sd_i: destination score)
    out_i += sum_j softmax_j(e_ij) z_j[head k]            (added in place into ``into``)

``z`` is this rank's transformed source rows, ``zh`` the halo rows — received by an
all-to-all-v of ``z``'s send rows started inside the op (hidden layers), or given
(``zh_static``: layer 0 transforms its kept halo feature rows itself, no exchange) — and
the two are read as two sources by the kernels (never concatenated). GPU: the three
kernels of csrc/kernels/gat_f32.hip (forward with on-the-fly softmax weights; backward
destination side; backward source side over the transposed pattern, which also carries
the ``a_src`` term into ``dz``); the halo rows' gradient returns to their owners through the
reverse all-to-all-v and is segment-summed there. CPU: the same math in plain PyTorch
autograd at fp64 (the numerics oracle).

Reference: experiments/OGB-LSC/RGAT.py:108-206 (per-edge gathers, concat, a linear layer,
exp without max subtraction, scatter-sum denominator: ~8 passes over E x C memory, and five
collectives per relation-layer).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch.autograd import Function

from .. import _native
from . import kernels as K
from .csr import CSR

SLOPE = 0.2
# GPU: one kernel pass per head over that head's columns (D = C / heads of 64/128/256)
# instead of whole rows — the SpMM's narrow-pass idea (kernels/spmm_f32.hip: a D-column
# slice of the neighbour rows keeps its locality window in the L2 / Infinity Cache longer).
# Measured on the 1/8 MAG240M RGAT step (4 heads, C = 256): the three attention kernels take
# 660 ms per step with head passes against 510 ms with whole rows (the per-pass softmax
# statistics, index reads and 4-rows-per-wave degree imbalance cost more than the locality
# gains; profiles/r06/rgat_eighth_kernels_per_step*.txt), so whole rows are the default;
# DGRAPH_GAT_HEAD_PASSES=1 selects the passes.
import os as _os

HEAD_PASSES = _os.environ.get("DGRAPH_GAT_HEAD_PASSES", "0") == "1"


def _passes(C: int, Hh: int):
    """[(column slice, head slice)] of the kernel calls of one op, and the heads per call."""
    D = C // Hh
    if HEAD_PASSES and Hh > 1 and D in (64, 128, 256):
        return [(slice(k * D, (k + 1) * D), slice(k, k + 1)) for k in range(Hh)], 1
    return [(slice(None), slice(None))], Hh


class GatPattern:
    """One relation's destination-row pattern over ``[local sources | halo rows]`` (int32
    columns, halo columns at ``nsplit + h``) and its transpose (source rows -> destination
    ids), built once per relation."""

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, nsplit: int, n_halo: int):
        self.rowptr = rowptr.long().contiguous()
        self.col = col.to(torch.int32).contiguous()
        self.nsplit, self.H = int(nsplit), int(n_halo)
        self.R = self.rowptr.numel() - 1
        ncols = self.nsplit + self.H
        if self.col.numel() and (int(self.col.min()) < 0 or int(self.col.max()) >= ncols):
            raise ValueError("GatPattern: a column id outside [0, local + halo)")
        from ..parallel.hetero_graph import _transpose_noperm

        t = _transpose_noperm(CSR(self.rowptr, self.col, ncols))
        self.t_rowptr = t.rowptr.long().contiguous()
        self.t_col = t.col.to(torch.int32).contiguous()

    @staticmethod
    def merged(interior: CSR, halo: Optional[CSR], nsplit: int) -> "GatPattern":
        """Each row's interior entries then its halo entries (shifted by ``nsplit``)."""
        if halo is None or halo.nnz == 0:
            H = 0 if halo is None else int(halo.num_cols)
            return GatPattern(interior.rowptr, interior.col, nsplit, H)
        dev = interior.device
        di = interior.rowptr[1:] - interior.rowptr[:-1]
        rp = interior.rowptr + halo.rowptr
        col = torch.empty(int(rp[-1]), dtype=torch.int32, device=dev)
        for part, first, shift in ((interior, None, 0), (halo, di, nsplit)):
            if part.nnz == 0:
                continue
            rows = part.row_ids()
            pos = rp[rows] + torch.arange(part.nnz, device=dev) - part.rowptr[rows]
            if first is not None:
                pos += first[rows]
            col[pos] = part.col.to(torch.int32) + shift
            del rows, pos
        return GatPattern(rp, col, nsplit, int(halo.num_cols))


def _score_matrix(a_src: torch.Tensor) -> torch.Tensor:
    """[heads, D] -> the block-diagonal [C, heads] matrix with ``z @ A = per-head z . a``."""
    Hh, D = a_src.shape
    A = a_src.new_zeros(Hh * D, Hh)
    for k in range(Hh):
        A[k * D:(k + 1) * D, k] = a_src[k]
    return A


def head_scores(z: torch.Tensor, a_src: torch.Tensor) -> torch.Tensor:
    """``s[n, k] = z[n, kD:(k+1)D] . a_src[k]`` (one [C, heads] GEMM, no [N, C] temporary)."""
    if z.shape[0] == 0:
        return z.new_zeros(0, a_src.shape[0])
    return (z @ _score_matrix(a_src.to(z.dtype))).contiguous()


def _reference(z, zh, sd, a_src, pat: GatPattern):
    """The relation's attention output [R, C], differentiable plain PyTorch (CPU oracle)."""
    Hh, D = a_src.shape
    zall = torch.cat([z, zh], 0) if zh is not None else z
    ss = head_scores(zall, a_src)
    rows = torch.repeat_interleave(torch.arange(pat.R), pat.rowptr[1:] - pat.rowptr[:-1])
    cols = pat.col.long()
    e = torch.nn.functional.leaky_relu(sd[rows] + ss[cols], SLOPE)  # [E, Hh]
    m = torch.full((pat.R, Hh), -float("inf"), dtype=e.dtype).index_reduce(
        0, rows, e.detach(), "amax", include_self=True)
    p = torch.exp(e - m[rows])
    den = torch.zeros(pat.R, Hh, dtype=e.dtype).index_add(0, rows, p)
    alpha = p / den[rows]
    msg = (zall[cols].view(-1, Hh, D) * alpha.unsqueeze(-1)).reshape(-1, Hh * D)
    return torch.zeros(pat.R, Hh * D, dtype=z.dtype).index_add(0, rows, msg)


class _GatRelFn(Function):
    @staticmethod
    def forward(ctx, z, zh_static, sd, a_src, into, pat: GatPattern, sg, heads: int,
                remake=None):
        Hh = int(heads)
        ctx.remake = remake
        exchange = zh_static is None and sg is not None and sg.halo is not None
        ctx.pat, ctx.sg, ctx.exchange, ctx.heads = pat, sg, exchange, Hh
        ctx.static = zh_static is not None
        if not z.is_cuda:
            with torch.enable_grad():
                zz = z.detach().double().requires_grad_()
                zhh = None
                if exchange:
                    zhh = sg.a2a(K.gather_rows(z.detach(), sg.send_map.idx)).double()
                elif zh_static is not None:
                    zhh = zh_static.detach().double()
                if zhh is not None:
                    zhh.requires_grad_()
                sdd = sd.detach().double().requires_grad_()
                aa = a_src.detach().double().requires_grad_()
                out = _reference(zz, zhh, sdd, aa, pat)
            ctx.cpu = (zz, zhh, sdd, aa, out)
            into.add_(out.detach().to(into.dtype))
            ctx.mark_dirty(into)
            return into
        ctx.cpu = None
        zh, work = zh_static, None
        if exchange:
            zh, work = sg.a2a(K.gather_rows(z, sg.send_map.idx), async_op=True)
        ss = head_scores(z, a_src)  # (overlaps the exchange)
        if work is not None:
            work.wait()
        ssh = head_scores(zh, a_src) if zh is not None and zh.shape[0] else None
        if ssh is None:
            zh = None
        R = pat.R
        m = torch.empty(R, Hh, dtype=torch.float32, device=z.device)
        l = torch.empty_like(m)
        sdc = sd.contiguous()
        passes, hp = _passes(z.shape[1], Hh)
        for cs, hs in passes:
            _native.ops().gat_fwd_f32(pat.rowptr, pat.col, z[:, cs],
                                      None if zh is None else zh[:, cs], pat.nsplit,
                                      ss[:, hs], None if ssh is None else ssh[:, hs],
                                      sdc[:, hs], into[:, cs], 1.0, m[:, hs], l[:, hs], hp,
                                      SLOPE)
        # remake = (x, W[, xh]): z (and a static zh) are x W^T — rebuilt bitwise in backward
        # by the same GEMM instead of being kept (x: the resident input features)
        # (an exchanged zh is received again in backward from the owners' rebuilt z)
        keep_z = z if remake is None else None
        keep_zh = zh if (remake is None or (zh_static is not None and len(remake) < 3)) \
            else None
        ctx.zh_remade = keep_zh is None and zh is not None
        ctx.save_for_backward(keep_z, keep_zh, ss, ssh, sd, m, l, a_src)
        ctx.mark_dirty(into)
        return into

    @staticmethod
    def backward(ctx, g):
        if ctx.cpu is not None:
            zz, zhh, sdd, aa, out = ctx.cpu
            ins = [t for t in (zz, zhh, sdd, aa) if t is not None]
            grads = torch.autograd.grad(out, ins, g.double(), allow_unused=True,
                                        retain_graph=True)  # (gradcheck re-enters)
            it = iter(grads)
            gz = next(it)
            gzh = next(it) if zhh is not None else None
            gsd, ga = next(it), next(it)
            z_dt = g.dtype
            gz = gz.to(z_dt)
            if ctx.exchange and gzh is not None:
                sg = ctx.sg
                back = sg.a2a_rev(gzh.to(z_dt).contiguous())
                st = sg.send_map.transpose_csr()
                K.spmm(st.rowptr, st.col, back, gz, beta=1.0)
                gzh = None
            return (gz, gzh.to(z_dt) if (gzh is not None and ctx.static) else None,
                    gsd.to(z_dt), ga.to(z_dt), g, None, None, None, None)
        z, zh, ss, ssh, sd, m, l, a_src = ctx.saved_tensors
        if ctx.remake is not None:
            from . import f32 as F32

            x, W = ctx.remake[0], ctx.remake[1]
            if z is None:
                z = F32.linear_fwd(x, W)
            if ctx.zh_remade:
                if ctx.exchange:  # every rank rebuilds its z here: the same rows again
                    zh = ctx.sg.a2a(K.gather_rows(z, ctx.sg.send_map.idx))
                else:
                    zh = F32.linear_fwd(ctx.remake[2], W)
        pat, Hh = ctx.pat, ctx.heads
        ops = _native.ops()
        g = g.contiguous()
        R, Ls = pat.R, z.shape[0]
        c = torch.empty(R, Hh, dtype=torch.float32, device=g.device)
        gsd = torch.empty_like(c)
        sdc = sd.contiguous()
        passes, hp = _passes(z.shape[1], Hh)
        for cs, hs in passes:
            ops.gat_bwd_dst_f32(pat.rowptr, pat.col, z[:, cs],
                                None if zh is None else zh[:, cs], pat.nsplit, ss[:, hs],
                                None if ssh is None else ssh[:, hs], sdc[:, hs], m[:, hs],
                                l[:, hs], g[:, cs], c[:, hs], gsd[:, hs], hp, SLOPE)
        a_flat = a_src.reshape(-1).contiguous()
        gz = torch.empty_like(z)
        gss = torch.empty(Ls, Hh, dtype=torch.float32, device=g.device)
        for cs, hs in passes:
            ops.gat_bwd_src_f32(pat.t_rowptr[:Ls + 1], pat.t_col, g[:, cs], z[:, cs],
                                ss[:, hs], sdc[:, hs], m[:, hs], l[:, hs], c[:, hs],
                                a_flat[cs], gz[:, cs], gss[:, hs], hp, SLOPE)
        Hh_, D = a_src.shape
        ga = (gss.t() @ z).view(Hh, Hh, D).diagonal(dim1=0, dim2=1).t()
        gzh = None
        if zh is not None:
            gzh = torch.empty_like(zh)
            gssh = torch.empty(zh.shape[0], Hh, dtype=torch.float32, device=g.device)
            for cs, hs in passes:
                ops.gat_bwd_src_f32(pat.t_rowptr[Ls:], pat.t_col, g[:, cs], zh[:, cs],
                                    ssh[:, hs], sdc[:, hs], m[:, hs], l[:, hs], c[:, hs],
                                    a_flat[cs], gzh[:, cs], gssh[:, hs], hp, SLOPE)
            ga = ga + (gssh.t() @ zh).view(Hh, Hh, D).diagonal(dim1=0, dim2=1).t()
            if ctx.exchange:
                # the halo rows' gradient back to their owners, summed there in a fixed order
                sg = ctx.sg
                back, work = sg.a2a_rev(gzh, async_op=True)
                work.wait()
                st = sg.send_map.transpose_csr()
                K.spmm(st.rowptr, st.col, back, gz, beta=1.0)
                gzh = None
        return (gz, gzh if ctx.static else None, gsd, ga.contiguous(), g, None, None, None,
                None)


def gat_relation_into(z: torch.Tensor, sd: torch.Tensor, a_src: torch.Tensor,
                      into: torch.Tensor, pat: GatPattern, sg=None,
                      zh_static: Optional[torch.Tensor] = None, remake=None) -> torch.Tensor:
    """``into += attention(z [, halo rows], sd, a_src)`` over ``pat`` (autograd; returns the
    updated ``into``). ``a_src``: [heads, D]. Halo rows: ``zh_static`` when given, else
    exchanged through ``sg`` (a :class:`~dgraph_amd.parallel.hetero_graph.SourceGraph`).
    ``remake = (x, W[, xh])`` (GPU): ``z = x W^T`` (and ``zh_static = xh W^T``) are
    recomputed in backward by the same exact-f32 GEMM instead of being saved — the layer-0
    memory diet (x: resident features)."""
    heads = a_src.shape[0]
    if z.is_cuda and z.dtype == torch.float32:
        C = z.shape[1]
        if C not in (64, 128, 256) or C % heads or (C // 4) // heads < 2:
            raise ValueError(f"gat_relation_into: unsupported width {C} / heads {heads}")
    if remake is not None and not z.is_cuda:
        remake = None  # (the CPU oracle keeps its own fp64 graph)
    return _GatRelFn.apply(z.contiguous(), zh_static, sd, a_src.contiguous(), into, pat, sg,
                           int(heads), remake)
