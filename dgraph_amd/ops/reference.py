"""Pure-PyTorch fp32 reference implementations of the native ops.

Used (a) for CPU tensors, so the whole framework runs and is tested without a GPU, and
(b) as the numerics oracle the HIP kernels are compared against in ``tests/``.
Semantics match :mod:`dgraph_amd.ops.kernels` exactly (see csrc/kernels/kernels.h).
"""
from __future__ import annotations

from typing import Optional

import torch


def _row_ids(rowptr: torch.Tensor) -> torch.Tensor:
    deg = rowptr[1:] - rowptr[:-1]
    return torch.repeat_interleave(torch.arange(deg.numel(), device=rowptr.device), deg)


def spmm(
    rowptr: torch.Tensor,
    col: torch.Tensor,
    x: torch.Tensor,
    out: torch.Tensor,
    edge_weight: Optional[torch.Tensor] = None,
    col_scale: Optional[torch.Tensor] = None,
    row_scale: Optional[torch.Tensor] = None,
    heads: int = 1,
    beta: float = 0.0,
    cap: int = 0,
) -> torch.Tensor:
    """``cap > 0``: every row sums only its first ``cap`` entries (hub-split main pass)."""
    R = rowptr.numel() - 1
    F = x.shape[1]
    col = col.long()
    rows = _row_ids(rowptr)
    keep = None
    if cap > 0 and col.numel() > 0:
        slot = torch.arange(col.numel(), device=col.device) - rowptr[:-1].long()[rows]
        keep = slot < cap
        col, rows = col[keep], rows[keep]
        if edge_weight is not None:
            edge_weight = edge_weight.reshape(keep.numel(), -1)[keep]
    adt = torch.float64 if x.dtype == torch.float64 else torch.float32
    vals = x.to(adt)[col]
    if edge_weight is not None:
        w = edge_weight.to(adt).reshape(col.numel(), max(heads, 1))
        hd = F // max(heads, 1)
        vals = (vals.view(-1, max(heads, 1), hd) * w.unsqueeze(-1)).view(-1, F)
    if col_scale is not None:
        vals = vals * col_scale.to(adt)[col].unsqueeze(1)
    acc = torch.zeros(R, F, dtype=adt, device=x.device)
    acc.index_add_(0, rows, vals)
    if row_scale is not None:
        acc = acc * row_scale.to(adt).unsqueeze(1)
    if beta != 0.0:
        acc = acc + beta * out[:R].to(adt)
    out[:R].copy_(acc.to(out.dtype))
    return out


def spmm_hub_partials(seg_beg, seg_end, col, x, partials, edge_weight=None, col_scale=None):
    """fp32 sums of the hub-tail segments ``col[seg_beg[i]:seg_end[i]]`` (cf. kernels.h;
    fp64 for fp64 inputs, so gradcheck sees the split path at full precision)."""
    cdt = torch.float64 if x.dtype == torch.float64 else torch.float32
    lens = seg_end - seg_beg
    S = seg_beg.numel()
    if S == 0:
        return partials
    seg = torch.repeat_interleave(torch.arange(S, device=col.device), lens)
    off = torch.zeros(S + 1, dtype=torch.long, device=col.device)
    torch.cumsum(lens, 0, out=off[1:])
    pos = seg_beg[seg] + (torch.arange(seg.numel(), device=col.device) - off[:-1][seg])
    c = col.long()[pos]
    vals = x.to(cdt)[c]
    w = torch.ones(pos.numel(), dtype=cdt, device=col.device)
    if edge_weight is not None:
        w = w * edge_weight.reshape(-1).to(cdt)[pos]
    if col_scale is not None:
        w = w * col_scale.to(cdt)[c]
    acc = torch.zeros(S, x.shape[1], dtype=cdt, device=x.device)
    acc.index_add_(0, seg, vals * w.unsqueeze(1))
    partials[:S].copy_(acc)
    return partials


def spmm_hub_reduce(partials, hub_seg_ptr, hub_rows, out, row_scale=None):
    """``out[hub_rows[h]] += row_scale * sum of the hub's segment partials`` (in order)."""
    nh = hub_rows.numel()
    if nh == 0:
        return out
    cnt = hub_seg_ptr[1:] - hub_seg_ptr[:-1]
    cdt = torch.float64 if out.dtype == torch.float64 else torch.float32
    owner = torch.repeat_interleave(torch.arange(nh, device=out.device), cnt)
    acc = torch.zeros(nh, out.shape[1], dtype=cdt, device=out.device)
    acc.index_add_(0, owner, partials[: owner.numel()].to(cdt))
    if row_scale is not None:
        acc = acc * row_scale.to(cdt)[hub_rows].unsqueeze(1)
    out[hub_rows] = (out[hub_rows].to(cdt) + acc).to(out.dtype)
    return out


def copy_rows(
    x: torch.Tensor,
    src_idx: Optional[torch.Tensor],
    dst_idx: Optional[torch.Tensor],
    out: torch.Tensor,
    accumulate: bool = False,
) -> torch.Tensor:
    n = (src_idx.numel() if src_idx is not None else
         dst_idx.numel() if dst_idx is not None else x.shape[0])
    if src_idx is not None:
        s = src_idx.long()
        vals = torch.zeros(n, x.shape[1], dtype=x.dtype, device=x.device)
        ok = s >= 0
        vals[ok] = x[s[ok]]
    else:
        vals = x[:n]
    if dst_idx is not None:
        d = dst_idx.long()
        keep = d >= 0
        d, vals = d[keep], vals[keep]
    else:
        d = torch.arange(n, device=x.device)
    if accumulate:
        out.index_add_(0, d, vals.to(out.dtype))
    else:
        out[d] = vals.to(out.dtype)
    return out


def masked_gather_rows(x, idx, mask, value, out):
    sel = mask == value
    out[sel] = x[idx[sel]]
    return out


def edge_softmax_fwd(rowptr: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    cdt = torch.float64 if s.dtype == torch.float64 else torch.float32
    s2 = s.to(cdt).reshape(s.shape[0], -1)
    rows = _row_ids(rowptr)
    R = rowptr.numel() - 1
    H = s2.shape[1]
    m = torch.full((R, H), float("-inf"), device=s.device, dtype=cdt)
    m = m.scatter_reduce(0, rows.unsqueeze(1).expand(-1, H), s2, reduce="amax")
    e = torch.exp(s2 - m[rows])
    den = torch.zeros(R, H, device=s.device, dtype=cdt).index_add_(0, rows, e)
    return (e / den[rows]).reshape(s.shape)


def edge_softmax_bwd(rowptr: torch.Tensor, alpha: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    cdt = torch.float64 if alpha.dtype == torch.float64 else torch.float32
    a2 = alpha.to(cdt).reshape(alpha.shape[0], -1)
    g2 = g.to(cdt).reshape(a2.shape)
    rows = _row_ids(rowptr)
    R = rowptr.numel() - 1
    dot = torch.zeros(R, a2.shape[1], device=alpha.device, dtype=cdt).index_add_(0, rows,
                                                                              a2 * g2)
    return (a2 * (g2 - dot[rows])).reshape(alpha.shape)


def _mask_to_words(keep: torch.Tensor) -> torch.Tensor:
    """Keep-mask -> int32 words in the kernels' layout: 512-element chunks, word j (64
    bit, little-endian int32 pair) of a chunk holds bit l = keep(8*l + j)."""
    flat = keep.reshape(-1)
    n = flat.numel()
    nch = (n + 511) // 512
    pad = torch.zeros(nch * 512, dtype=torch.bool, device=flat.device)
    pad[:n] = flat
    k = pad.view(nch, 64, 8).permute(0, 2, 1).to(torch.int64)  # [chunk, j, lane]
    lo = (k[:, :, :32] << torch.arange(32, device=k.device)).sum(-1)
    hi = (k[:, :, 32:] << torch.arange(32, device=k.device)).sum(-1)
    w = torch.stack([lo, hi], -1).reshape(-1)
    w = torch.where(w >= 2**31, w - 2**32, w)
    return w.to(torch.int32)


def _words_to_mask(bits: torch.Tensor, numel: int) -> torch.Tensor:
    nch = (numel + 511) // 512
    w = bits.reshape(-1)[: nch * 16].to(torch.int64) & 0xFFFFFFFF
    w = w.view(nch, 8, 2)
    lanes = torch.arange(32, device=w.device)
    lo = (w[:, :, 0:1] >> lanes) & 1
    hi = (w[:, :, 1:2] >> lanes) & 1
    k = torch.cat([lo, hi], -1)  # [chunk, j, lane]
    return k.permute(0, 2, 1).reshape(-1)[:numel].bool()


def bias_relu_pack(y: torch.Tensor, bias, bits, relu: bool) -> None:
    t = y.float()
    if bias is not None:
        t = t + bias.float()
    if relu:
        keep = t > 0
        t = torch.where(keep, t, torch.zeros((), device=t.device))
        if bits is not None:
            w = _mask_to_words(keep)
            bits.view(-1)[: w.numel()] = w
    y.copy_(t.to(y.dtype))


def relu_mask_bwd(g: torch.Tensor, bits: torch.Tensor) -> None:
    keep = _words_to_mask(bits, g.numel()).reshape(g.shape)
    g.masked_fill_(~keep, 0)


def row_scale_cols(x: torch.Tensor, s: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    out.copy_((x.float() * s.float().unsqueeze(1)).to(out.dtype))
    return out


def row_scale_colsum(x: torch.Tensor, s: torch.Tensor, out: torch.Tensor,
                     partial: torch.Tensor) -> torch.Tensor:
    nb = partial.shape[0]
    rpb = (x.shape[0] + nb - 1) // nb
    xf = x.float()
    partial.zero_()
    for b in range(nb):
        partial[b] = xf[b * rpb:(b + 1) * rpb].sum(0)
    return row_scale_cols(x, s, out)


def col_sum(g: torch.Tensor) -> torch.Tensor:
    return g.float().sum(0)


def pair_relu(rowptr, col, mode: int, rowterm, gat, gat2=None, rowmul=None, out=None):
    """CPU reference of the fused edge-MLP aggregation (csrc/kernels/edge_fused.hip)."""
    cdt = torch.float64 if gat.dtype == torch.float64 else torch.float32
    R = rowptr.numel() - 1
    rows = _row_ids(rowptr)
    c = col.long()
    pre = rowterm.to(cdt)[rows] + gat.to(cdt)[c]
    if mode == 0:
        val = pre.clamp_min(0)
    elif mode == 1:
        val = (pre > 0).to(cdt)
    else:
        val = torch.where(pre > 0, gat2.to(cdt)[c], torch.zeros((), dtype=cdt))
    acc = torch.zeros(R, gat.shape[1], dtype=cdt).index_add_(0, rows, val)
    if mode == 1:
        acc = acc * rowmul.to(cdt)[:R]
    if out is None:
        return acc.to(gat.dtype)
    out[:R].copy_(acc)
    return out


def _act(x, act: int):
    if act == 1:
        return x.clamp_min(0)
    if act == 2:
        return x * torch.sigmoid(x)
    if act == 3:
        return torch.where(x > 0, x, 0.2 * x)
    return x


def _act_grad(x, act: int):
    if act == 1:
        return (x > 0).to(x.dtype)
    if act == 2:
        s = torch.sigmoid(x)
        return s * (1 + x * (1 - s))
    if act == 3:
        return torch.where(x > 0, torch.ones_like(x), torch.full_like(x, 0.2))
    return torch.ones_like(x)


def gather_add_act(Y, P, src, Q, dst, gin, out, act: int):
    cdt = torch.float64 if out.dtype == torch.float64 else torch.float32
    E, F = out.shape
    pre = torch.zeros(E, F, dtype=cdt)
    if Y is not None:
        pre += Y[:E].to(cdt)
    if P is not None:
        pre += P.to(cdt)[src[:E].long()]
    if Q is not None:
        pre += Q.to(cdt)[dst[:E].long()]
    if gin is None:
        out.copy_(_act(pre, act))
    else:
        out.copy_(gin[:E].to(cdt) * _act_grad(pre, act))
    return out


def tile32_encode(keep: torch.Tensor) -> torch.Tensor:
    """Keep mask [M, N] -> int64 words in the dual-GEMM "tile32" layout
    (csrc/kernels/dual_gemm.hip): word[(rb * NT + t) * 16 + r] bit l = keep of
    (32 rb + (r & 3) + 8 (r >> 2) + 4 (l >> 5), 32 t + (l & 31)); rows padded to 256."""
    M, N = keep.shape
    NT = N // 32
    Mp = (M + 255) // 256 * 256
    k = torch.zeros(Mp, N, dtype=torch.bool)
    k[:M] = keep.cpu()
    lane = torch.arange(64)
    r = torch.arange(16)
    rows = (r.unsqueeze(1) & 3) + 8 * (r.unsqueeze(1) >> 2) + 4 * (lane.unsqueeze(0) >> 5)  # [16, 64]
    cols = lane & 31
    kt = k.view(Mp // 32, 32, NT, 32)                      # [rb, rr, t, cc]
    # non-adjacent advanced indices: the broadcast index dims come first -> [16, 64, rb, t]
    bits = kt[:, rows, :, cols.unsqueeze(0).expand(16, 64)]
    bits = bits.permute(2, 3, 0, 1).to(torch.int64)        # [rb, t, 16, 64]
    w = (bits << torch.arange(64, dtype=torch.int64)).sum(-1)  # wraps like uint64
    return w.reshape(-1)


def tile32_decode(words: torch.Tensor, M: int, N: int) -> torch.Tensor:
    NT = N // 32
    Mp = (M + 255) // 256 * 256
    w = words.cpu()[: Mp // 32 * NT * 16].view(Mp // 32, NT, 16, 1)
    bits = ((w >> torch.arange(64, dtype=torch.int64)) & 1).bool()  # [rb, t, 16, 64]
    lane = torch.arange(64)
    r = torch.arange(16)
    rows = (r.unsqueeze(1) & 3) + 8 * (r.unsqueeze(1) >> 2) + 4 * (lane.unsqueeze(0) >> 5)
    cols = (lane & 31).unsqueeze(0).expand(16, 64)
    out = torch.zeros(Mp // 32, 32, NT, 32, dtype=torch.bool)
    out[:, rows, :, cols] = bits.permute(2, 3, 0, 1)  # -> [16, 64, rb, t]
    return out.view(Mp, N)[:M]
