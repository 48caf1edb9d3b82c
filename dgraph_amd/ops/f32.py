"""fp32 (reference-precision) compute ops: device dispatch.

GPU tensors -> hand-written gfx950 kernels (``csrc/kernels/{spmm_f32,gemm_f32,wgrad_f32,
bits}.hip``); CPU tensors -> plain-PyTorch fp64-accumulated references (the numerics oracle
of the tests, and the path the gloo multi-process tests run). No GPU fallback: a missing
native library raises (:func:`dgraph_amd._native.ops`).

The reference is fp32-only (DGraph/distributed/csrc/torch_local_kernels.cu:43-46); these
ops are what :mod:`dgraph_amd.models.sage_fused` is built from.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _native


# ------------------------------------------------------------------------------ SpMM

def spmm_f32(rowptr: torch.Tensor, col: torch.Tensor, x: torch.Tensor,
             out: Optional[torch.Tensor] = None, *, row_scale=None, col_scale=None,
             edge_weight=None, col_map: Optional[torch.Tensor] = None,
             row_ids: Optional[torch.Tensor] = None, beta: float = 0.0,
             row_map: Optional[torch.Tensor] = None,
             gate: Optional[torch.Tensor] = None, self_add: Optional[torch.Tensor] = None,
             self_map: Optional[torch.Tensor] = None, self_row0: int = 0,
             pass_cols: int = 0, rowend: Optional[torch.Tensor] = None,
             x2: Optional[torch.Tensor] = None, nsplit: int = 0) -> torch.Tensor:
    """``out[o(i)] = row_scale[o(i)] * sum_j w_j X(m(col_j)) + beta * out[o(i)]`` over the
    entries of CSR row ``r = row_ids[i]`` (all rows when None): ``[rowptr[r], rowptr[r+1])``,
    or ``[rowptr[r], rowend[r])`` when ``rowend`` is given (one run of a row stored in two);
    ``m = col_map`` (entries with ``col_map < 0`` skipped) or identity; ``X(c) = x[c]``, or
    with ``x2`` (two sources in one pass) ``x2[c - nsplit]`` for ``c >= nsplit``; ``o =
    row_map`` or identity. ``gate`` (indexed like ``out``): the stored value is kept where
    ``gate > 0`` (a ReLU derivative). ``self_add``: output row o also gets
    ``self_add[self_map[self_row0 + o]]`` (when >= 0), before the gate. ``pass_cols`` (GPU):
    the column-pass width of this call (0 = the process default, 64): narrow passes keep a
    locality window in the caches, full-width passes make each random row access one long
    read (see FusedSAGE's autotune)."""
    if row_ids is not None:
        n = row_ids.numel()
    else:
        n = rowend.numel() if rowend is not None else rowptr.numel() - 1
    if out is None:
        if row_map is not None:
            raise ValueError("spmm_f32: row_map needs an explicit out")
        out = torch.empty(n, x.shape[1], dtype=x.dtype, device=x.device)
        beta = 0.0
    if x.is_cuda:
        _native.ops().spmm_f32_ex(rowptr, col, edge_weight, col_scale, row_scale, col_map,
                                  row_ids, x, out, float(beta), 0, row_map, gate, self_add,
                                  self_map, int(self_row0), rowend, x2, int(nsplit),
                                  int(pass_cols))
        return out
    # CPU reference (fp64 accumulation)
    rp = rowptr.long()
    nr = rowend.numel() if rowend is not None else rp.numel() - 1
    rows = torch.arange(nr, device=rp.device) if row_ids is None else row_ids.long()
    beg = rp[rows]
    end = rowend.long()[rows] if rowend is not None else rp[rows + 1]
    deg = end - beg
    seg = torch.repeat_interleave(torch.arange(n, device=rp.device), deg)
    off = torch.zeros(n + 1, dtype=torch.long, device=rp.device)
    torch.cumsum(deg, 0, out=off[1:])
    pos = beg[seg] + (torch.arange(seg.numel(), device=rp.device) - off[:-1][seg])
    c = col.long()[pos]
    w = torch.ones(c.numel(), dtype=torch.float64)
    if edge_weight is not None:
        w = w * edge_weight.double()[pos]
    if col_map is not None:
        c = col_map.long()[c]
        keep = c >= 0
        w = torch.where(keep, w, torch.zeros_like(w))
        c = torch.where(keep, c, torch.zeros_like(c))
    if col_scale is not None:
        w = w * col_scale.double()[c]
    acc = torch.zeros(n, x.shape[1], dtype=torch.float64)
    if c.numel():
        if x2 is not None:
            lo = c < nsplit
            rows_x = torch.empty(c.numel(), x.shape[1], dtype=torch.float64)
            rows_x[lo] = x.double()[c[lo]]
            rows_x[~lo] = x2.double()[c[~lo] - nsplit]
        else:
            rows_x = x.double()[c]
        acc.index_add_(0, seg, rows_x * w.unsqueeze(1))
    o = torch.arange(n) if row_map is None else row_map.long()
    if row_scale is not None:
        acc = acc * row_scale.double()[o].unsqueeze(1)
    if beta != 0.0:
        acc = acc + beta * out[o].double()
    if self_add is not None:
        m = self_map.long()[self_row0 + o]
        add = self_add.double()[m.clamp_min(0)][:, :acc.shape[1]]
        acc = acc + torch.where((m >= 0).unsqueeze(1), add, torch.zeros_like(add))
    if gate is not None:
        acc = torch.where(gate[o][:, :acc.shape[1]] > 0, acc, torch.zeros_like(acc))
    out[o] = acc.to(out.dtype)
    return out


# ------------------------------------------------------------------------------ GEMM
def gemm_f32_ok(N: int, K1: int, K2: int = 0) -> bool:
    return N in (64, 128, 176, 192, 256) and K1 % 32 == 0 and K1 > 0 and K2 % 32 == 0


def gemm_f32(A1: torch.Tensor, B1: torch.Tensor, A2=None, B2=None, *, a_rows=None, bias=None,
             cin=None, beta: float = 1.0, gate=None, o_rows=None, relu: bool = False,
             out: Optional[torch.Tensor] = None, row_scale=None) -> torch.Tensor:
    """``out[o(i)] = relu?(gate?(rs[i] (A1[a(i)] @ B1 (+ A2[i] @ B2)) + bias +
    beta*cin[o(i)]))`` (csrc/kernels/gemm_f32.hip; B row-major [K, N]); ``gate``: keep
    where gate > 0; ``row_scale`` (nullable [M]): per input row."""
    M = a_rows.numel() if a_rows is not None else A1.shape[0]
    N = B1.shape[1]
    if out is None:
        if o_rows is not None:
            raise ValueError("gemm_f32: o_rows needs an explicit out")
        out = torch.empty(M, N, dtype=torch.float32, device=A1.device)
    if A1.is_cuda:
        _native.ops().gemm_f32(A1, B1.contiguous(), A2, None if B2 is None else B2.contiguous(),
                               a_rows, None if bias is None else bias.float().contiguous(),
                               cin, float(beta), gate, o_rows, bool(relu), out,
                               None if row_scale is None else row_scale.float().contiguous())
        return out
    a = A1.double()[a_rows.long()] if a_rows is not None else A1[:M].double()
    v = a @ B1.double()
    if A2 is not None:
        v = v + A2[:M].double() @ B2.double()
    o = torch.arange(M) if o_rows is None else o_rows.long()
    if row_scale is not None:
        v = v * row_scale.double()[:M].unsqueeze(1)
    if bias is not None:
        v = v + bias.double()
    if cin is not None:
        v = v + beta * cin[o].double()
    if gate is not None:
        v = torch.where(gate[o][:, :N] > 0, v, torch.zeros_like(v))
    if relu:
        v = v.clamp_min(0)
    out[o] = v.to(out.dtype)
    return out


class WgradAcc:
    """``dW += [A1[a1_rows] | A2]^T G`` accumulated over calls (row chunks of one step) in
    per-unit fp32 partial slabs (csrc/kernels/wgrad_f32.hip: a call's rows are cut into
    units, one slab each, pulled dynamically by at most one block per CU), reduced once in
    a fixed order by :meth:`result` — deterministic for a fixed chunking. Two units per CU
    by default, so a CU held by another stream's kernel costs a share of one unit, not a
    whole block's."""

    UNITS_PER_CU = 2

    _P = 0

    def __init__(self, K: int, N: int, device, blocks: int = 0):
        self.K, self.N, self.device = int(K), int(N), torch.device(device)
        if self.device.type == "cuda":
            if blocks <= 0:
                if WgradAcc._P == 0:
                    WgradAcc._P = torch.cuda.get_device_properties(self.device).multi_processor_count
                blocks = WgradAcc._P * self.UNITS_PER_CU
            self.partials = torch.empty(blocks, self.K, self.N, dtype=torch.float32,
                                        device=self.device)
        else:
            self.partials = torch.zeros(1, self.K, self.N, dtype=torch.float64)
        self.fresh = True
        self.used = 0  # slabs written since reset

    # rows per block of a short call: fewer blocks -> fewer partial slabs read and
    # written, but each block's rows run serially (2048: a 1.4K-row call took 0.4 ms on
    # one CU; 64 spreads it over ~22)
    MIN_ROWS_PER_BLOCK = 64

    def reset(self):
        self.fresh = True
        self.used = 0

    def add(self, A1: torch.Tensor, G: torch.Tensor, A2: Optional[torch.Tensor] = None,
            a1_rows: Optional[torch.Tensor] = None) -> None:
        if G.shape[0] == 0:
            return
        if self.device.type == "cuda":
            P = self.partials.shape[0]
            nb = max(1, min(P, -(-G.shape[0] // self.MIN_ROWS_PER_BLOCK)))
            _native.ops().wgrad_f32(A1, A2, a1_rows, G, self.partials, nb, self.used)
            self.used = max(self.used, nb)
        else:
            M = G.shape[0]
            a = A1.double()[a1_rows.long()] if a1_rows is not None else A1[:M].double()
            if A2 is not None:
                a = torch.cat([a, A2[:M].double()], 1)
            p = a.t() @ G.double()
            if self.fresh:
                self.partials[0].copy_(p)
            else:
                self.partials[0] += p
        self.fresh = False

    def result(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if out is None:
            out = torch.empty(self.K, self.N, dtype=torch.float32, device=self.device)
        if self.fresh:
            return out.zero_()
        if self.device.type == "cuda":
            _native.ops().wgrad_f32_reduce(self.partials[: self.used], out)
        else:
            out.copy_(self.partials[0].to(out.dtype))
        return out


# ------------------------------------------------------------------------------ bits
def row_keep_bits(h: torch.Tensor, rows: Optional[torch.Tensor] = None,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """int32 [n, F/32] words: bit j of word w of row i = ``h[rows[i], 32w + j] > 0``."""
    n = rows.numel() if rows is not None else h.shape[0]
    W = h.shape[1] // 32
    if out is None:
        out = torch.empty(n, W, dtype=torch.int32, device=h.device)
    if h.is_cuda:
        _native.ops().row_keep_bits(h, rows, out)
        return out
    hr = h[rows.long()] if rows is not None else h[:n]
    b = (hr > 0).view(n, W, 32).long()
    sh = torch.arange(32, dtype=torch.long)
    words = (b << sh).sum(-1)
    out.copy_(((words + (1 << 31)) % (1 << 32) - (1 << 31)).to(torch.int32).view(n, W))
    return out


def apply_keep_bits(g: torch.Tensor, bits: torch.Tensor) -> torch.Tensor:
    """In place ``g[i, f] = bit(i, f) ? g[i, f] : 0``."""
    if g.is_cuda:
        _native.ops().apply_keep_bits(g, bits)
        return g
    n, F = g.shape
    w = bits.view(n, F // 32).long() & 0xFFFFFFFF
    keep = ((w.unsqueeze(-1) >> torch.arange(32, dtype=torch.long)) & 1).view(n, F).bool()
    g.mul_(keep.to(g.dtype))
    return g


# ------------------------------------------------------------------------------ loss
def xent_rows(z: torch.Tensor, rows: torch.Tensor, y: torch.Tensor, scale: float,
              dz: torch.Tensor, row_loss: torch.Tensor, C: int) -> None:
    """Softmax cross-entropy of logit rows ``z[rows[i], :C]`` with labels ``y``:
    ``row_loss[i] = lse - z_y``, ``dz[i, :C] = (softmax - onehot) * scale`` and
    ``dz[i, C:] = 0`` (csrc/kernels/loss.hip)."""
    n = rows.numel()
    if n == 0:
        return
    if z.is_cuda:
        _native.ops().xent_rows(z, rows, y, float(scale), dz, row_loss, int(C))
        return
    zt = z[rows.long()][:, :C].double()
    lse = torch.logsumexp(zt, 1)
    row_loss[:n] = (lse - zt.gather(1, y.long().unsqueeze(1)).squeeze(1)).to(row_loss.dtype)
    p = torch.exp(zt - lse.unsqueeze(1))
    p[torch.arange(n), y.long()] -= 1.0
    dz[:n].zero_()
    dz[:n, :C] = (p * scale).to(dz.dtype)


def argmax_hits(z: torch.Tensor, rows: torch.Tensor, y: torch.Tensor, hit: torch.Tensor,
                C: int) -> None:
    """``hit[i] = (argmax z[rows[i], :C] == y[i])`` (first maximum), uint8."""
    n = rows.numel()
    if n == 0:
        return
    if z.is_cuda:
        _native.ops().argmax_hits(z, rows, y, hit, int(C))
        return
    hit[:n] = (z[rows.long()][:, :C].argmax(1) == y.long()).to(hit.dtype)
