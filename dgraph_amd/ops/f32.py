"""fp32 (reference-precision) compute ops: device dispatch.

GPU tensors -> hand-written gfx950 kernels (``csrc/kernels/{spmm_f32,gemm_f32,wgrad_f32,
bits}.hip``); CPU tensors -> plain-PyTorch fp64-accumulated references (the numerics oracle
of the tests, and the path the gloo multi-process tests run). No GPU fallback: a missing
native library raises (:func:`dgraph_amd._native.ops`).

The reference is fp32-only (DGraph/distributed/csrc/torch_local_kernels.cu:43-46); these
ops are what :mod:`dgraph_amd.models.sage_fused` is built from.
"""
from __future__ import annotations

import os
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
             x2: Optional[torch.Tensor] = None, nsplit: int = 0,
             keep_bits: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``out[o(i)] = row_scale[o(i)] * sum_j w_j X(m(col_j)) + beta * out[o(i)]`` over the
    entries of CSR row ``r = row_ids[i]`` (all rows when None): ``[rowptr[r], rowptr[r+1])``,
    or ``[rowptr[r], rowend[r])`` when ``rowend`` is given (one run of a row stored in two);
    ``m = col_map`` (entries with ``col_map < 0`` skipped) or identity; ``X(c) = x[c]``, or
    with ``x2`` (two sources in one pass) ``x2[c - nsplit]`` for ``c >= nsplit``; ``o =
    row_map`` or identity. ``gate`` (indexed like ``out``): the stored value is kept where
    ``gate > 0`` (a ReLU derivative). ``self_add``: output row o also gets
    ``self_add[self_map[self_row0 + o]]`` (when >= 0), before the gate. ``keep_bits``
    ([out rows, F/32] int32, as ``row_keep_bits`` writes them): zero column c of output
    row o unless bit c of its words is set (a 1-bit ReLU derivative). ``pass_cols`` (GPU):
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
                                  int(pass_cols), keep_bits)
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
    if keep_bits is not None:
        acc = torch.where(unpack_keep_bits(keep_bits[o], acc.shape[1]), acc,
                          torch.zeros_like(acc))
    out[o] = acc.to(out.dtype)
    return out


def unpack_keep_bits(words: torch.Tensor, F: int) -> torch.Tensor:
    """[rows, W] int32 keep words -> [rows, F] bool (bit c of a row's words: column c)."""
    sh = torch.arange(32, device=words.device, dtype=torch.int32)
    return (((words.unsqueeze(2) >> sh) & 1) != 0).reshape(words.shape[0], -1)[:, :F]


# ------------------------------------------------------------------------------ GEMM
def gemm_f32_ok(N: int, K1: int, K2: int = 0) -> bool:
    return N in (64, 128, 176, 192, 256) and K1 % 32 == 0 and K1 > 0 and K2 % 32 == 0


def gemm_f32(A1: torch.Tensor, B1: torch.Tensor, A2=None, B2=None, *, a_rows=None, bias=None,
             cin=None, beta: float = 1.0, gate=None, o_rows=None, relu: bool = False,
             out: Optional[torch.Tensor] = None, row_scale=None, send=None) -> torch.Tensor:
    """``out[o(i)] = relu?(gate?(rs[i] (A1[a(i)] @ B1 (+ A2[i] @ B2)) + bias +
    beta*cin[o(i)]))`` (csrc/kernels/gemm_f32.hip; B row-major [K, N]); ``gate``: keep
    where gate > 0; ``row_scale`` (nullable [M]): per input row. ``send`` = (send_out
    [rows, N], send_ptr int64 [M + 1], send_pos int32): the halo pack fused into the
    producer — row i is also stored to send_out rows send_pos[send_ptr[i]:send_ptr[i + 1]]
    (not with o_rows)."""
    M = a_rows.numel() if a_rows is not None else A1.shape[0]
    N = B1.shape[1]
    if send is not None and o_rows is not None:
        raise ValueError("gemm_f32: send is not combined with o_rows")
    if out is None:
        if o_rows is not None:
            raise ValueError("gemm_f32: o_rows needs an explicit out")
        out = torch.empty(M, N, dtype=torch.float32, device=A1.device)
    if A1.is_cuda:
        B1 = B1.contiguous()
        B2 = None if B2 is None else B2.contiguous()
        bias = None if bias is None else bias.float().contiguous()
        rs = None if row_scale is None else row_scale.float().contiguous()
        ops = _native.ops()
        # N beyond one kernel tile (a 512-wide hidden layer): column blocks, A read per block
        blocks = [(0, N)] if N <= 256 else _blocks(N, lambda w: w in (128, 176, 192, 256))
        if len(blocks) > 1:
            # one kernel reads its A rows before it overwrites them (tile by tile), but a
            # later column block would read what an earlier one wrote: an A that shares
            # memory with out (the in-place boundary-row / streamed-halo GEMM of a wide
            # hidden layer) is copied once first
            if _overlaps(A1, out):
                A1 = A1.clone()
            if A2 is not None and _overlaps(A2, out):
                A2 = A2.clone()
        so, sp, sq = send if send is not None else (None, None, None)
        for n0, n1 in blocks:
            full = (n0, n1) == (0, N)
            ops.gemm_f32(A1, B1 if full else B1[:, n0:n1], A2,
                         None if B2 is None else (B2 if full else B2[:, n0:n1]), a_rows,
                         None if bias is None else bias[n0:n1], None if cin is None else
                         (cin if full else cin[:, n0:n1]), float(beta),
                         None if gate is None else (gate if full else gate[:, n0:n1]), o_rows,
                         bool(relu), out if full else out[:, n0:n1], rs,
                         None if so is None else (so if full else so[:, n0:n1]), sp, sq)
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
    if send is not None:
        so, sp, sq = send
        sp = sp.long()
        rows = torch.repeat_interleave(torch.arange(M, device=sp.device), sp[1:] - sp[:-1])
        q = torch.arange(int(sp[0]), int(sp[-1]), device=sp.device)
        so[sq.long()[q]] = v[rows].to(so.dtype)
    return out


def _span(t: torch.Tensor):
    """Byte range [lo, hi) a strided tensor's elements occupy."""
    if t.numel() == 0:
        return (0, 0)
    lo = t.data_ptr()
    hi = lo + (1 + sum((s - 1) * st for s, st in zip(t.shape, t.stride()))) * t.element_size()
    return (lo, hi)


def _overlaps(a: torch.Tensor, b: torch.Tensor) -> bool:
    if a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr():
        return False
    (a0, a1), (b0, b1) = _span(a), _span(b)
    return a0 < b1 and b0 < a1


def _wgrad_n_ok(n: int) -> bool:
    return n in (128, 176, 192, 256)


def _blocks(n: int, ok, widths=(256, 192, 176, 128)):
    """Cut ``n`` columns into blocks whose widths satisfy ``ok`` (greedy, widest first)."""
    out, c = [], 0
    while c < n:
        for w in widths:
            if n - c >= w and ok(w) and (n - c - w == 0 or n - c - w >= min(widths)):
                out.append((c, c + w))
                c += w
                break
        else:
            raise ValueError(f"no kernel block decomposition of {n} columns")
    return out


class _WgradTile:
    """One native accumulator: ``dW[K, N] += [A1[a1_rows] | A2]^T G`` for K in {128, 256},
    N in {128, 176, 192, 256} (csrc/kernels/wgrad_f32.hip: a call's rows are cut into
    units, one fp32 partial slab each, pulled dynamically by at most one block per CU),
    reduced once in unit order — deterministic for a fixed chunking."""

    def __init__(self, K: int, N: int, device, units: int, colsum: bool = False):
        self.K, self.N = K, N
        self.partials = torch.empty(units, K, N, dtype=torch.float32, device=device)
        # G's column sums per unit (a bias gradient), computed by the same kernel pass
        self.col = torch.empty(units, N, dtype=torch.float32, device=device) if colsum \
            else None
        self.used = 0

    def add(self, A1, G, A2, a1_rows, min_rows: int) -> None:
        P = self.partials.shape[0]
        nb = max(1, min(P, -(-G.shape[0] // min_rows)))
        _native.ops().wgrad_f32(A1, A2, a1_rows, G, self.partials, nb, self.used, self.col)
        self.used = max(self.used, nb)

    def result(self, out: torch.Tensor) -> torch.Tensor:
        _native.ops().wgrad_f32_reduce(self.partials[: self.used], out)
        return out

    def col_result(self, out: torch.Tensor) -> torch.Tensor:
        _native.ops().wgrad_f32_reduce(self.col[: self.used].unsqueeze(1), out)
        return out


class WgradAcc:
    """``dW += [A1[a1_rows] | A2]^T G`` accumulated over calls (row chunks of one step),
    deterministic for a fixed chunking (the fp32 weight gradients of the fused executors).

    GPU: native split-M MFMA accumulators (:class:`_WgradTile`); a ``[K, N]`` product wider
    than one kernel tile (K > 256: a wide input layer, ``[x | mean_N(x)]`` of a 768-wide
    feature; N > 256: a 512-wide hidden layer) is cut into K-blocks of the concatenated
    ``[A1 | A2]`` columns and N-blocks of G's columns, one accumulator each (G is read once
    per K-block); row units are pulled dynamically by the blocks. CPU: one fp64 accumulator
    (the numerics oracle). One row unit per CU by default (``DGRAPH_WGRAD_UNITS_PER_CU``): two cost 8 ms
    per papers100M step in slab traffic, and the kernel's blocks share a CU with another
    stream's waves without slowing down (profiles/r04/gemm_wgrad_static_vs_dynamic_ab.log)."""

    UNITS_PER_CU = int(os.environ.get("DGRAPH_WGRAD_UNITS_PER_CU", "1"))
    # rows per unit of a short call: fewer units -> fewer partial slabs read and written,
    # but each unit's rows run serially (2048: a 1.4K-row call took 0.4 ms on one CU; 64
    # spreads it over ~22)
    MIN_ROWS_PER_BLOCK = 64

    _P = 0

    def __init__(self, K: int, N: int, device, blocks: int = 0, colsum: bool = False):
        self.K, self.N, self.device = int(K), int(N), torch.device(device)
        self.fresh = True
        self.colsum = bool(colsum)
        self.tiles = []
        if self.device.type == "cuda":
            if blocks <= 0:
                if WgradAcc._P == 0:
                    WgradAcc._P = torch.cuda.get_device_properties(self.device).multi_processor_count
                blocks = WgradAcc._P * self.UNITS_PER_CU
            kb = _blocks(self.K, lambda w: w in (128, 256), (256, 128))
            nb = _blocks(self.N, _wgrad_n_ok)
            for k0, k1 in kb:
                for n0, n1 in nb:
                    # the column sums ride on the first K-block of every N-block
                    self.tiles.append(((k0, k1), (n0, n1),
                                       _WgradTile(k1 - k0, n1 - n0, self.device, blocks,
                                                  colsum=self.colsum and k0 == 0)))
        else:
            self.partials = torch.zeros(1, self.K, self.N, dtype=torch.float64)
            self.cols = torch.zeros(self.N, dtype=torch.float64)

    def reset(self):
        self.fresh = True
        for t in self.tiles:
            t[2].used = 0

    def add(self, A1: torch.Tensor, G: torch.Tensor, A2: Optional[torch.Tensor] = None,
            a1_rows: Optional[torch.Tensor] = None) -> None:
        if G.shape[0] == 0:
            return
        if self.device.type == "cuda":
            K1 = A1.shape[1] if A2 is not None else self.K
            if A2 is None and A1.shape[1] != self.K:
                A1 = A1[:, : self.K]
            for (k0, k1), (n0, n1), t in self.tiles:
                g = G if (n0, n1) == (0, G.shape[1]) else G[:, n0:n1]
                if k1 <= K1:  # A1 columns only (rows through a1_rows)
                    a = A1 if (k0, k1) == (0, A1.shape[1]) else A1[:, k0:k1]
                    t.add(a, g, None, a1_rows, self.MIN_ROWS_PER_BLOCK)
                elif k0 >= K1:  # A2 columns only (dense rows)
                    t.add(A2[:, k0 - K1:k1 - K1], g, None, None, self.MIN_ROWS_PER_BLOCK)
                else:  # straddles: the kernel's dual form
                    t.add(A1[:, k0:K1], g, A2[:, : k1 - K1], a1_rows, self.MIN_ROWS_PER_BLOCK)
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
            if self.colsum:
                cs = G.double().sum(0)
                if self.fresh:
                    self.cols.copy_(cs)
                else:
                    self.cols += cs
        self.fresh = False

    def col_result(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Column sums of every G added since the last reset (``colsum=True``): the bias
        gradient that goes with the weight gradient, from the same kernel pass."""
        if not self.colsum:
            raise ValueError("WgradAcc: built without colsum")
        if out is None:
            out = torch.empty(self.N, dtype=torch.float32, device=self.device)
        if self.fresh:
            return out.zero_()
        if self.device.type == "cuda":
            for (k0, k1), (n0, n1), t in self.tiles:
                if k0 == 0:
                    if (n0, n1) == (0, self.N):
                        t.col_result(out)
                    else:
                        blk = torch.empty(n1 - n0, dtype=torch.float32, device=self.device)
                        out[n0:n1] = t.col_result(blk)
        else:
            out.copy_(self.cols.to(out.dtype))
        return out

    def result(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if out is None:
            out = torch.empty(self.K, self.N, dtype=torch.float32, device=self.device)
        if self.fresh:
            return out.zero_()
        if self.device.type == "cuda":
            if len(self.tiles) == 1 and out.is_contiguous():
                self.tiles[0][2].result(out)
                return out
            for (k0, k1), (n0, n1), t in self.tiles:
                blk = torch.empty(k1 - k0, n1 - n0, dtype=torch.float32, device=self.device)
                out[k0:k1, n0:n1] = t.result(blk)
        else:
            out.copy_(self.partials[0].to(out.dtype))
        return out


# ------------------------------------------------------------------------------ Linear
# ``y = x W^T + b`` layers (torch Linear layout, W: [N, K]) at fp32 on the kernels above,
# for any model's linears (ops.dense.linear / linear_sum, ops.act_linear): the library fp32
# GEMM is the fallback for widths the kernels do not tile (e.g. 153 classes) and for
# non-fp32 / CPU tensors. Switch: DGRAPH_F32_LINEAR=0 -> library GEMMs everywhere.
LINEAR_ON = os.environ.get("DGRAPH_F32_LINEAR", "1") != "0"


def tileable(n: int) -> bool:
    """Output widths the fp32 GEMM covers (one tile, or 128/176/192/256 column blocks)."""
    if gemm_f32_ok(n, 32):
        return True
    try:
        _blocks(n, lambda w: w in (128, 176, 192, 256))
        return n > 256
    except ValueError:
        return False


def wgrad_ok(K: int, N: int) -> bool:
    try:
        _blocks(K, lambda w: w in (128, 256), (256, 128))
        _blocks(N, _wgrad_n_ok)
        return True
    except ValueError:
        return False


def _on(*ts) -> bool:
    return LINEAR_ON and all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 2
                             and t.stride(1) == 1 and t.shape[0] > 0 for t in ts)


def linear_fwd(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor] = None):
    """``x W^T + b``."""
    N, K = W.shape
    if _on(x) and K % 32 == 0 and tileable(N):
        return gemm_f32(x, W.t().contiguous(), bias=b)
    return torch.nn.functional.linear(x, W.to(x.dtype), None if b is None else b.to(x.dtype))


def linear_dgrad(gs, Ws) -> torch.Tensor:
    """``sum_i g_i W_i`` (two terms per kernel call, the running sum chained through
    ``cin``). Narrow terms (an output width that is not a multiple of 32, e.g. the per-head
    attention scores of RGAT's destination projection) are packed side by side into ONE
    zero-padded 32-wide term of the same chain, instead of sending the whole sum to the
    library GEMM."""
    K = Ws[0].shape[1]
    gs = [g if g.stride(-1) == 1 else g.contiguous() for g in gs]
    if _on(*gs) and tileable(K):
        big = [(g, W) for g, W in zip(gs, Ws) if g.shape[1] % 32 == 0]
        small = [(g, W) for g, W in zip(gs, Ws) if g.shape[1] % 32 != 0]
        if small:
            n = sum(g.shape[1] for g, _ in small)
            npad = _pad32(n)
            gcat = gs[0].new_zeros(gs[0].shape[0], npad)
            Wcat = Ws[0].new_zeros(npad, K)
            off = 0
            for g, W in small:
                w = g.shape[1]
                gcat[:, off:off + w] = g
                Wcat[off:off + w] = W.to(Wcat.dtype)
                off += w
            big.append((gcat, Wcat))
        out = None
        for k in range(0, len(big), 2):
            two = k + 1 < len(big)
            out = gemm_f32(big[k][0], big[k][1].contiguous(), big[k + 1][0] if two else None,
                           big[k + 1][1].contiguous() if two else None, cin=out, out=out)
        return out
    out = gs[0] @ Ws[0].to(gs[0].dtype)
    for g, W in zip(gs[1:], Ws[1:]):
        out = out + g @ W.to(g.dtype)
    return out


def _pad32(n: int) -> int:
    return (n + 31) // 32 * 32


def wgrad_tiled(g: torch.Tensor, x: torch.Tensor, W: torch.Tensor) -> bool:
    """Does :func:`linear_wgrad` run the MFMA accumulator for this shape (else None)?"""
    N, K = W.shape
    return _on(g, x) and wgrad_ok(K, N)


def linear_wgrad(g: torch.Tensor, x: torch.Tensor, W: torch.Tensor, bias: bool = False):
    """``g^T x`` in W's layout [N, K] (split-M MFMA accumulator), or None when the kernels
    do not tile the shape (callers then use their own library path). ``bias``: returns
    ``(dW, g.sum(0))``, the column sums from the same kernel pass."""
    N, K = W.shape
    if _on(g, x) and wgrad_ok(K, N):
        acc = WgradAcc(K, N, g.device, colsum=bias)
        acc.add(x, g)
        dW = acc.result().t().contiguous().to(W.dtype)
        return (dW, acc.col_result()) if bias else dW
    return None


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


def apply_keep_bits(g: torch.Tensor, bits: torch.Tensor,
                    rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """In place ``g[i, f] = bit(i, f) ? g[i, f] : 0`` (for the rows ``rows`` only, bits
    indexed by the same row, when given)."""
    if g.is_cuda:
        _native.ops().apply_keep_bits(g, bits, rows)
        return g
    n, F = g.shape
    w = bits.view(n, F // 32).long() & 0xFFFFFFFF
    if rows is not None:
        r = rows.long()
        keep = ((w[r].unsqueeze(-1) >> torch.arange(32, dtype=torch.long)) & 1).view(
            r.numel(), F).bool()
        g[r] = g[r] * keep.to(g.dtype)
        return g
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
