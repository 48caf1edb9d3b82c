"""Functional entry points of the native op library (device dispatch).

GPU tensors -> hand-written HIP kernels in ``csrc/kernels`` (via ``torch.ops.dgraph_amd``);
CPU tensors -> :mod:`dgraph_amd.ops.reference`. There is no GPU fallback: a missing
native library raises (see :func:`dgraph_amd._native.ops`).

Native-kernel counterparts of the reference's ``torch_local`` module
(DGraph/distributed/csrc/torch_local_kernels.cu:28-254), generalised to bf16/fp32,
int32/int64 indices and wave64.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _native
from . import reference as _ref


def _native_ok(t: torch.Tensor) -> bool:
    return t.is_cuda


def _f32(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if t is None:
        return None
    if t.dtype != torch.float32 or not t.is_contiguous():
        t = t.float().contiguous()
    return t


def spmm(
    rowptr: torch.Tensor,
    col: torch.Tensor,
    x: torch.Tensor,
    out: Optional[torch.Tensor] = None,
    *,
    edge_weight: Optional[torch.Tensor] = None,
    col_scale: Optional[torch.Tensor] = None,
    row_scale: Optional[torch.Tensor] = None,
    heads: int = 1,
    beta: float = 0.0,
    split=None,
    row_map: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """CSR aggregation ``out[r] = row_scale[r]*sum_j w_j*col_scale[c_j]*x[c_j] + beta*out[r]``.

    ``split``: a :class:`~dgraph_amd.ops.csr.HubSplit` of this CSR (one head only): hub
    rows sum their first ``split.cap`` entries in the main pass and their tails in
    independent segment waves, added back in a fixed order (same result; no wave is held
    by a 10^5-degree row).

    ``row_map``: CSR row r is output row ``row_map[r]`` (a row-compacted CSR,
    :meth:`~dgraph_amd.ops.csr.CSR.compact_rows`); ``out`` must then be given."""
    R = rowptr.numel() - 1
    F = x.shape[1]
    if row_map is not None and out is None:
        raise ValueError("spmm: row_map needs an explicit out")
    if out is None:
        out = torch.empty(R, F, dtype=x.dtype, device=x.device)
        beta = 0.0
    heads = max(int(heads), 1)
    if split is not None and heads != 1:
        split = None
    cap = split.cap if split is not None else 0
    ew, cs, rs = _f32(edge_weight), _f32(col_scale), _f32(row_scale)
    if _native_ok(x):
        ops = _native.ops()
        ops.spmm(rowptr, col, ew, cs, rs, x, out, heads, F // heads, float(beta), cap,
                 row_map)
        if split is not None:
            part = torch.empty(split.num_segments, F, dtype=torch.float32, device=x.device)
            ops.spmm_hub_partials(split.seg_beg, split.seg_end, col, ew, cs, x, part)
            ops.spmm_hub_reduce(part, split.hub_seg_ptr, split.hub_rows, rs, out)
        return out
    if row_map is not None:
        rs_c = None if row_scale is None else row_scale[row_map]
        tmp = out[row_map] if beta != 0.0 else torch.empty(R, F, dtype=out.dtype,
                                                            device=out.device)
        _ref.spmm(rowptr, col, x, tmp, edge_weight, col_scale, rs_c, heads, beta, cap)
        out[row_map] = tmp
    else:
        _ref.spmm(rowptr, col, x, out, edge_weight, col_scale, row_scale, heads, beta, cap)
    if split is not None:
        pdt = torch.float64 if x.dtype == torch.float64 else torch.float32
        part = torch.empty(split.num_segments, F, dtype=pdt, device=x.device)
        _ref.spmm_hub_partials(split.seg_beg, split.seg_end, col, x, part, edge_weight,
                               col_scale)
        _ref.spmm_hub_reduce(part, split.hub_seg_ptr, split.hub_rows, out, row_scale)
    return out


def copy_rows(
    x: torch.Tensor,
    src_idx: Optional[torch.Tensor] = None,
    dst_idx: Optional[torch.Tensor] = None,
    out: Optional[torch.Tensor] = None,
    *,
    num_out_rows: Optional[int] = None,
    accumulate: bool = False,
) -> torch.Tensor:
    """``out[dst[i]] (+)= x[src[i]]`` (identity when an index is None)."""
    if out is None:
        n = (src_idx.numel() if src_idx is not None else x.shape[0])
        rows = num_out_rows if num_out_rows is not None else n
        alloc = torch.zeros if (accumulate or dst_idx is not None) else torch.empty
        out = alloc(rows, x.shape[1], dtype=torch.float32 if accumulate else x.dtype,
                    device=x.device)
    if src_idx is not None and dst_idx is not None and src_idx.dtype != dst_idx.dtype:
        src_idx, dst_idx = src_idx.long(), dst_idx.long()
    if _native_ok(x):
        xin = x.float() if (accumulate and x.dtype != torch.float32) else x
        _native.ops().copy_rows(xin, src_idx, dst_idx, out, bool(accumulate))
        return out
    return _ref.copy_rows(x, src_idx, dst_idx, out, accumulate)


def gather_rows(x: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """``out[i] = x[idx[i]]`` (zeros where idx < 0)."""
    out = torch.empty(idx.numel(), x.shape[1], dtype=x.dtype, device=x.device)
    return copy_rows(x, src_idx=idx, out=out)


def masked_gather_rows(x, idx, mask, value, out):
    if _native_ok(x):
        _native.ops().masked_gather_rows(x, idx.long(), mask.long(), int(value), out)
        return out
    return _ref.masked_gather_rows(x, idx, mask, value, out)


def edge_softmax_fwd(rowptr: torch.Tensor, scores: torch.Tensor) -> torch.Tensor:
    if _native_ok(scores):
        s = scores.float().contiguous()
        alpha = torch.empty_like(s)
        _native.ops().edge_softmax_fwd(rowptr, s, alpha)
        return alpha
    return _ref.edge_softmax_fwd(rowptr, scores)


def edge_softmax_bwd(rowptr: torch.Tensor, alpha: torch.Tensor, grad: torch.Tensor) -> torch.Tensor:
    if _native_ok(alpha):
        a = alpha.float().contiguous()
        g = grad.float().contiguous()
        ds = torch.empty_like(a)
        _native.ops().edge_softmax_bwd(rowptr, a, g, ds)
        return ds
    return _ref.edge_softmax_bwd(rowptr, alpha, grad)


def mask_words(numel: int) -> int:
    """int32 words of a keep mask for ``numel`` elements (512-element chunks x 16)."""
    return (numel + 511) // 512 * 16


def col_sum(g: torch.Tensor) -> torch.Tensor:
    """fp32 column sums of a 2-D tensor (bias gradients), deterministic."""
    if _native_ok(g) and g.dim() == 2 and g.stride(1) == 1:
        vec = 4 if g.dtype == torch.float32 else 8
        if g.shape[1] % vec != 0 or g.stride(0) % vec != 0:
            vec = 1  # scalar-lane kernel variant
        if g.shape[1] // vec <= 256:
            return _native.ops().col_sum(g)
        return torch.sum(g, dim=0, dtype=torch.float32)
    return _ref.col_sum(g)


def row_scale_colsum(x: torch.Tensor, s: torch.Tensor, out: torch.Tensor,
                     partial: torch.Tensor) -> torch.Tensor:
    """:func:`row_scale_cols` (bf16) that also writes fp32 column sums of the UNSCALED
    ``x`` over a fixed row partition into ``partial [nblocks, w]`` (may be a column slice
    of a wider partials tensor); ``partial.sum(0)`` are the column sums. Native: one
    pass (elementwise.hip row_scale_colsum)."""
    if _native_ok(x):
        _native.ops().row_scale_colsum(x, _f32(s), out, partial)
        return out
    return _ref.row_scale_colsum(x, s, out, partial)


def row_scale_cols(x: torch.Tensor, s: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """``out[r, :] = x[r, :] * s[r]`` for a row-strided ``x`` (e.g. a column slice);
    fp32 ``s``. Native: one streaming pass with 16-B lanes (elementwise.hip)."""
    if _native_ok(x):
        _native.ops().row_scale_cols(x, _f32(s), out)
        return out
    return _ref.row_scale_cols(x, s, out)


def bias_relu_pack(y: torch.Tensor, bias: Optional[torch.Tensor] = None,
                   bits: Optional[torch.Tensor] = None, relu: bool = True) -> None:
    """In place ``y = act(y + bias)``; optional 1-bit keep mask (int32 words)."""
    if _native_ok(y):
        _native.ops().bias_relu_pack(y, _f32(bias), bits, bool(relu))
        return
    _ref.bias_relu_pack(y, bias, bits, relu)


def relu_mask_bwd(g: torch.Tensor, bits: torch.Tensor) -> None:
    """In place ``g = keep ? g : 0`` from a mask written by :func:`bias_relu_pack`."""
    if _native_ok(g):
        _native.ops().relu_mask_bwd(g, bits)
        return
    _ref.relu_mask_bwd(g, bits)


def pair_relu(rowptr: torch.Tensor, col: torch.Tensor, mode: int, rowterm: torch.Tensor,
              gat: torch.Tensor, gat2: Optional[torch.Tensor] = None,
              rowmul: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused edge-MLP aggregation (edge_fused.hip). mode 0: ``sum_c relu(R[r]+X[c])``;
    1: ``M[r] * #{R[r]+X[c] > 0}``; 2: ``sum_c X2[c] [R[r]+X[c] > 0]``."""
    R = rowptr.numel() - 1
    if out is None:
        out = torch.empty(R, gat.shape[1], dtype=gat.dtype, device=gat.device)
    if _native_ok(gat):
        _native.ops().pair_relu(rowptr, col, int(mode), rowterm, gat, gat2, rowmul, out)
        return out
    return _ref.pair_relu(rowptr, col, mode, rowterm, gat, gat2, rowmul, out)


ACT_IDS = {None: 0, "none": 0, "identity": 0, "relu": 1, "silu": 2, "leaky_relu": 3}


def gather_add_act(E: int, F: int, *, Y=None, P=None, src=None, Q=None, dst=None, gin=None,
                   act="none", out: Optional[torch.Tensor] = None,
                   dtype=None, device=None) -> torch.Tensor:
    """``out[e] = act(Y[e] + P[src[e]] + Q[dst[e]])``; with ``gin``: ``gin[e] * act'(...)``."""
    ref = next(t for t in (Y, P, Q, gin, out) if t is not None)
    if out is None:
        out = torch.empty(E, F, dtype=dtype or ref.dtype, device=device or ref.device)
    a = ACT_IDS[act]
    if _native_ok(out):
        _native.ops().gather_add_act(Y, P, src, Q, dst, gin, out, a)
        return out
    return _ref.gather_add_act(Y, P, src, Q, dst, gin, out, a)
