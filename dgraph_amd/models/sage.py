"""GraphSAGE (mean aggregator) for vertex-partitioned full-graph training.

The north-star model of BASELINE.json (ogbn-papers100M-shaped 3-layer GraphSAGE). The
reference has no GraphSAGE; this is built on the library's
distributed aggregation (:mod:`dgraph_amd.parallel.dist_graph`).

Each layer is ONE autograd node, designed for the 288 GB HBM budget of a single MI355X
holding a 111M-vertex / 3.2B-edge graph:

    y = act(x @ W_self + mean_{j in N(i)} x_j @ W_neigh + b)

* aggregation runs at ``min(F_in, F_out)`` features: aggregate-then-project when
  F_in <= F_out, project-then-aggregate otherwise (linearity);
* the aggregate is *not* stored for backward unless memory allows (``save_agg``); it is
  recomputed by one more SpMM, so a layer saves nothing beyond its input and output,
  which the neighbouring layers hold anyway;
* weights are fp32 masters, compute is bf16 with fp32 accumulation; weight gradients are
  produced in fp32 directly by the GEMM (``out_dtype``) where supported.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as Fn
from torch.autograd import Function

from .. import _native
from ..ops import kernels as K
from ..parallel import halo_recompute as _hr
from ..ops.dense import (col_sum_f32, dual_gemm, dual_gemm_shape_ok, mm_f32,  # noqa: F401
                         tile32_mask_words, wgrad)
from ..parallel.dist_graph import DistGraph


class SAGELayerFn(Function):
    @staticmethod
    def forward(ctx, x, w_self, w_neigh, bias, graph: DistGraph, relu: bool,
                project_first: bool, save_agg: bool):
        dt = x.dtype
        ws, wn = w_self.to(dt), w_neigh.to(dt)
        a_saved = None
        if project_first:
            z = x @ wn
            y = graph.aggregate(z, mean=True)
            del z
            if bias is not None:
                y.add_(bias.to(dt))
            y.addmm_(x, ws)
        else:
            a = graph.aggregate(x, mean=True)
            y = torch.addmm(bias.to(dt), x, ws) if bias is not None else x @ ws
            y.addmm_(a, wn)
            if save_agg:
                a_saved = a
            del a
        if relu:
            y.relu_()
        ctx.graph, ctx.relu, ctx.project_first = graph, relu, project_first
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, y if relu else None, ws, wn, a_saved)
        ctx.w_dtype = w_self.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y, ws, wn, a = ctx.saved_tensors
        graph: DistGraph = ctx.graph
        g = gy.to(x.dtype)
        if ctx.relu:
            g = torch.where(y > 0, g, torch.zeros((), dtype=g.dtype, device=g.device))
        g = g.contiguous()
        dws = wgrad(x, g).to(ctx.w_dtype) if ctx.needs_input_grad[1] else None
        db = col_sum_f32(g).to(ctx.w_dtype) if ctx.has_bias and ctx.needs_input_grad[3] else None
        dx = dwn = None
        if ctx.project_first:
            dz = graph.aggregate_T(g, mean=True)
            if ctx.needs_input_grad[2]:
                dwn = wgrad(x, dz).to(ctx.w_dtype)
            if ctx.needs_input_grad[0]:
                dx = g @ ws.t()
                dx.addmm_(dz, wn.t())
            del dz
        elif ctx.needs_input_grad[0] and a is None and wn.shape[1] <= 2 * wn.shape[0]:
            # one SpMM at F_out: u = A^T g -> dW_neigh = x^T u, dx = g Ws^T + u Wn^T
            u = graph.aggregate_T(g, mean=True)
            if ctx.needs_input_grad[2]:
                dwn = wgrad(x, u).to(ctx.w_dtype)
            dx = g @ ws.t()
            dx.addmm_(u, wn.t())
            del u
        else:
            if ctx.needs_input_grad[2]:
                if a is None:
                    a = graph.aggregate(x, mean=True)
                dwn = wgrad(a, g).to(ctx.w_dtype)
                del a
            if ctx.needs_input_grad[0]:
                t = g @ wn.t()
                dx = graph.aggregate_T(t, mean=True)
                del t
                dx.addmm_(g, ws.t())
        return dx, dws, dwn, db, None, None, None, None


class SAGEConv(nn.Module):
    """One GraphSAGE-mean layer over a :class:`DistGraph`."""

    def __init__(self, in_dim: int, out_dim: int, bias: bool = True, relu: bool = True,
                 order: str = "auto", save_agg: Optional[bool] = None):
        super().__init__()
        self.in_dim, self.out_dim, self.relu = in_dim, out_dim, relu
        self.w_self = nn.Parameter(torch.empty(in_dim, out_dim))
        self.w_neigh = nn.Parameter(torch.empty(in_dim, out_dim))
        self.bias = nn.Parameter(torch.zeros(out_dim)) if bias else None
        if order not in ("auto", "aggregate_first", "project_first"):
            raise ValueError(order)
        self.order = order
        self.save_agg = save_agg
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.w_self)
        nn.init.xavier_uniform_(self.w_neigh)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def project_first(self) -> bool:
        if self.order == "auto":
            return self.out_dim < self.in_dim
        return self.order == "project_first"

    def forward(self, x: torch.Tensor, graph: DistGraph) -> torch.Tensor:
        save = self.save_agg
        if save is None:
            save = _auto_save_agg(x, graph)
        return SAGELayerFn.apply(x, self.w_self, self.w_neigh, self.bias, graph, self.relu,
                                 self.project_first(), bool(save))


def _auto_save_agg(x: torch.Tensor, graph: DistGraph) -> bool:
    """Store the aggregate for backward only if it costs < 15% of free device memory."""
    if not x.is_cuda:
        return True
    free, _ = torch.cuda.mem_get_info(x.device)
    return x.numel() * x.element_size() < 0.15 * free


def _pad8(n: int) -> int:
    return (n + 7) // 8 * 8


def _pad_width(n: int) -> int:
    """Storage width of a hidden/output activation. Multiples of 8 give 16-B vector rows;
    when it costs <= 12 % more elements the width is rounded to 64 (128-B rows): a row
    that straddles cache lines makes the gather-bound SpMM fetch partial lines (a 352-B
    row at F=176 touches 3.5 lines on average, measured 4.8 vs 6.0 TB/s effective at F=128
    on the papers100M shape)."""
    p64 = (n + 63) // 64 * 64
    return p64 if p64 - n <= 0.12 * n else _pad8(n)


def _padded(params, i, dims_p, dt):
    """Layer i's (W_self, W_neigh, bias) cast to ``dt`` and zero-padded to
    ``[dims_p[i], dims_p[i+1]]`` (bias stays fp32 for the fused epilogue)."""
    ws, wn, b = params[3 * i], params[3 * i + 1], params[3 * i + 2]
    ri, ro = dims_p[i] - ws.shape[0], dims_p[i + 1] - ws.shape[1]
    if ri or ro:
        ws = Fn.pad(ws, (0, ro, 0, ri))
        wn = Fn.pad(wn, (0, ro, 0, ri))
        if b is not None:
            b = Fn.pad(b, (0, ro))
    return ws.to(dt), wn.to(dt), b


class SageWorkspace:
    """Preplanned activation slots for :class:`SAGEStackFn` (no per-step allocation).

    Slot plan for dims ``d_0..d_n`` over ``L`` rows (bf16):
      act[i]  (i = 1..n-1): hidden activation h_i, later its gradient dh_i (recycled)
      tmp_a               : aggregate / projection temp of every layer (fwd) and the
                            dense output gradient + aggregate recompute (bwd)
      tmp_b               : last-layer output (fwd) and aggregate_T temp (bwd)
    For the papers100M shape this is 209 GB of slots + 28 GB of features + 14 GB of CSR:
    the steady state performs no device allocation at all. (The caching allocator freed
    and re-mapped tens-of-GB blocks every step — 1.6 s of hipFree/hipMalloc per block on
    MI355X — measured with rocprofv3, profiles/.)
    """

    def __init__(self):
        self.key = None
        self.slots = {}
        self.generation = 0

    # device memory that must stay free after the optional ``agg0`` slot (RCCL buffers,
    # masks, weight-gradient partials and allocator slack)
    AGG0_HEADROOM = 24 << 30

    def prepare(self, L: int, dims, pf_flags, dtype, device, keep_agg0: bool = False,
                rows0: Optional[int] = None):
        """``rows0``: rows of the first layer's output and aggregate when they exceed
        ``L`` (halo recomputation: owned + padding + halo rows)."""
        rows0 = L if rows0 is None else int(rows0)
        key = (L, tuple(dims), tuple(pf_flags), dtype, str(device), keep_agg0, rows0)
        if key == self.key:
            return
        self.slots = {}
        n = len(dims) - 1
        C = dims[-1]
        wa = max([C] + [(dims[i + 1] if pf_flags[i] else dims[i]) for i in range(n)])
        wb = max([C] + [dims[i + 1] for i in range(n) if pf_flags[i]])
        for i in range(1, n):
            self.slots[f"act{i}"] = torch.empty((rows0 if i == 1 else L) * dims[i],
                                                dtype=dtype, device=device)
        na = L * wa
        if rows0 > L:  # layer-0 aggregate and layer-1 u over the extended rows
            na = max(na, rows0 * max(dims[0], dims[2] if n > 2 else 0))
        self.slots["tmp_a"] = torch.empty(na, dtype=dtype, device=device)
        self.slots["tmp_b"] = torch.empty(L * wb, dtype=dtype, device=device)
        if keep_agg0 and not pf_flags[0]:
            # layer 0's aggregate A x0 kept for its weight gradient (saves one SpMM per
            # step) when it fits next to the other slots (multi-GPU shards; not 1-GPU
            # papers100M, which needs ~263 GB without it)
            need = rows0 * dims[0] * torch.empty((), dtype=dtype).element_size()
            free = torch.cuda.mem_get_info(device)[0] if torch.device(device).type == "cuda" \
                else need + (64 << 30)  # host memory: treated as ample
            if free - need >= self.AGG0_HEADROOM:
                self.slots["agg0"] = torch.empty(rows0 * dims[0], dtype=dtype, device=device)
        self.key = key

    def mask(self, i: int, words: int, device) -> torch.Tensor:
        """Layer ``i``'s 1-bit ReLU mask words (persistent: a 3.5 GB-per-layer allocation
        per step at the papers100M shape otherwise, which at ~271 GB makes the caching
        allocator release and re-map blocks once anything else grows)."""
        name = f"mask{i}"
        buf = self.slots.get(name)
        if buf is None or buf.numel() < words or buf.device != torch.device(device):
            self.slots.pop(name, None)
            buf = torch.empty(words, dtype=torch.int64, device=device)
            self.slots[name] = buf
        return buf[:words]

    def has(self, name: str) -> bool:
        return name in self.slots

    def view(self, name: str, L: int, F: int) -> torch.Tensor:
        return self.slots[name][: L * F].view(L, F)


def _fusable(t: torch.Tensor, N: int, K1: int, K2: int = 0) -> bool:
    """Can the native MFMA dual GEMM (csrc/kernels/dual_gemm.hip) run this combine?"""
    return (t.is_cuda and t.dtype == torch.bfloat16 and _native.available()
            and dual_gemm_shape_ok(N, K1, K2))


def _bwd_fused(specs, dims_p, i: int, need_dx: bool, t: torch.Tensor) -> bool:
    """Layer i's input gradient is produced by one dual GEMM (pf: g Ws^T + dz Wn^T;
    aggregate-first with the u-trick: g Ws^T + u Wn^T) — so it can also apply the
    previous layer's ReLU mask in its epilogue."""
    _, pf = specs[i]
    if not need_dx:
        return False
    if not pf and dims_p[i + 1] > 2 * dims_p[i]:
        return False
    return _fusable(t, dims_p[i], dims_p[i + 1], dims_p[i + 1])


class SAGEStackFn(Function):
    """The whole layer stack as ONE autograd node (memory-lean training path).

    Owning every hidden activation lets backward *recycle* buffers: after layer i's weight
    gradients are formed from its input ``h_i``, ``h_i``'s storage receives ``dh_i``; ReLU
    layers keep a 1-bit mask instead of their output; all large tensors live in the
    preplanned :class:`SageWorkspace` slots. Peak for the papers100M shape on one GPU:
    ~251 GB of 288 GB (per-layer autograd would need ~330 GB).
    """

    @staticmethod
    def forward(ctx, x0, graph: DistGraph, specs, out_rows, ws_obj, restrict_last,
                eval_rows, *params):
        """Returns ``(logits[out_rows] or all logits, logits[eval_rows])``; the second output
        is not differentiable (validation/test predictions from the SAME forward, as the
        reference's epoch does, experiments/OGB/main.py:140-184).

        ``restrict_last``: with ``out_rows`` and a project-first output layer, aggregate
        only the loss rows in that layer (A[rows, :] z) instead of all vertices. Exact for
        the returned rows, but the other vertices get no logits, so it is incompatible with
        ``eval_rows`` and is NOT a full-graph forward (bench.py reports it separately)."""
        # workspace slots are used on the training path (row-subset output); a full
        # output must own its storage, so that path allocates
        use_ws = ws_obj is not None and out_rows is not None
        if restrict_last and eval_rows is not None:
            raise ValueError("restrict_last computes only the loss rows; eval_rows need the "
                             "full output layer")
        n = len(specs)
        L = x0.shape[0]
        dt = x0.dtype
        dims = [x0.shape[1]] + [params[3 * i].shape[1] for i in range(n)]
        # hidden/output widths padded to multiples of 8 (16-B bf16 rows: full-width
        # vector loads in the SpMM and the ReLU-mask kernels); pads stay exactly zero
        dims_p = [dims[0]] + [_pad_width(d) for d in dims[1:]]
        pf_flags = [pf for (_, pf) in specs]
        # halo recomputation (parallel/halo_recompute.py): layer 0 runs on the owned AND
        # halo rows, layer 1 reads its halo rows locally (no exchange either way)
        rc = getattr(graph, "recompute", None)
        if rc is not None and not (n >= 3 and not pf_flags[0] and not pf_flags[1]
                                   and not x0.requires_grad and out_rows is not None
                                   and dims_p[2] <= 2 * dims_p[1]):
            rc = None
        L1 = rc.L1 if rc is not None else L
        if use_ws:
            ws_obj.prepare(L, dims_p, pf_flags, dt, x0.device,
                           keep_agg0=not x0.requires_grad, rows0=L1)
            ws_obj.generation += 1
        keep0 = use_ws and ws_obj.has("agg0") and not pf_flags[0] and not x0.requires_grad
        V = (lambda name, F: ws_obj.view(name, L, F)) if use_ws else \
            (lambda name, F: torch.empty(L, F, dtype=dt, device=x0.device))
        V1 = (lambda name, F: ws_obj.view(name, L1, F)) if use_ws else \
            (lambda name, F: torch.empty(L1, F, dtype=dt, device=x0.device))
        acts = [x0]
        masks = []
        h = x0
        X_ext = None
        if rc is not None:
            X_ext = rc.inputs(x0)
            h = X_ext[:L1]
            acts = [h]
        for i, (relu, pf) in enumerate(specs):
            ws, wn, b = _padded(params, i, dims_p, dt)
            ws_, wn_ = ws, wn
            last = i == n - 1
            Fi, Fo = dims_p[i], dims_p[i + 1]
            rows_i = L1 if (rc is not None and i == 0) else L
            y = (V1 if rows_i != L else V)("tmp_b" if last else f"act{i + 1}", Fo)
            # one MFMA dual GEMM for the whole combine (+ bias, ReLU, 1-bit mask) when the
            # shape is supported and, for a ReLU layer, the backward consumer of its mask
            # (layer i + 1's input-gradient GEMM) is fused too (same "tile32" mask layout)
            fused = _fusable(h, Fo, Fi, 0 if pf else Fi) and (
                not relu or (i + 1 < n and _bwd_fused(specs, dims_p, i + 1, True, h)))
            mask = None
            if fused and relu:
                words = tile32_mask_words(rows_i, Fo)
                mask = ws_obj.mask(i, words, h.device) if use_ws else \
                    torch.empty(words, dtype=torch.int64, device=h.device)
            if last and pf and not relu and out_rows is not None and restrict_last:
                # only the loss rows leave the node: y[rows] = A[rows, :] (h Wn) +
                # h[rows] Ws + b — the row-restricted SpMM reads ~|rows|/L of the edges
                # and receives only the halo rows those rows touch
                z = torch.mm(h, wn_, out=V("tmp_a", Fo))
                y_rows = graph.aggregate_rows(z, out_rows, mean=True)
                del z
                if b is not None:
                    y_rows.add_(b.to(dt))
                y_rows.addmm_(h.index_select(0, out_rows), ws_)
                masks.append(None)
                h = y_rows
                break
            if pf:
                z = V("tmp_a", Fo)
                if fused:  # the projection on the same streaming MFMA kernel
                    dual_gemm(h, wn_.t().contiguous(), out=z)
                else:
                    torch.mm(h, wn_, out=z)
                graph.aggregate(z, mean=True, out=y)
                del z
                if fused:
                    dual_gemm(h, ws_.t().contiguous(), bias=b, cin=y, out=y, relu=relu,
                              mask_out=mask)
                else:
                    y.addmm_(h, ws_)
            else:
                slot = "agg0" if (i == 0 and keep0) else "tmp_a"
                if rc is not None and i == 0:
                    a = rc.aggregate0(X_ext, V1(slot, Fi))
                elif rc is not None and i == 1:
                    # the halo rows of h1 were computed here: no exchange
                    if _hr.MERGED:
                        a = rc.aggregate_owned(h, V(slot, Fi))
                    else:
                        a = graph.aggregate(h[:L], mean=True, out=V(slot, Fi),
                                            halo_rows=h[rc.Lp:rc.L1])
                    h = h[:L]
                else:
                    # layer 0 aggregates the input features: read-only without grad, so
                    # their halo rows are exchanged once and kept (DistGraph._static_halo)
                    a = graph.aggregate(h, mean=True, out=V(slot, Fi),
                                        static=i == 0 and not x0.requires_grad)
                if fused:
                    dual_gemm(h, ws_.t().contiguous(), a, wn_.t().contiguous(), bias=b, out=y,
                              relu=relu, mask_out=mask)
                else:
                    torch.mm(h, ws_, out=y)
                    y.addmm_(a, wn_)
                del a
            if fused:
                masks.append(("t32", mask) if relu else None)
            elif relu and Fo % 8 == 0 and y.is_contiguous():
                bits = torch.empty(K.mask_words(y.numel()), dtype=torch.int32, device=y.device)
                K.bias_relu_pack(y, b, bits, relu=True)
                masks.append(bits)
            else:
                if b is not None:
                    y.add_(b.to(dt))
                if relu:
                    y.relu_()
                masks.append(y if relu else None)
            if not last:
                acts.append(y)
            h = y
        ctx.graph, ctx.specs, ctx.dims, ctx.dims_p = graph, specs, dims, dims_p
        ctx.acts, ctx.masks = acts, masks
        ctx.x0_requires_grad = x0.requires_grad
        ctx.ws, ctx.use_ws, ctx.keep0 = ws_obj, use_ws, keep0
        ctx.rc, ctx.X_ext = rc, X_ext
        ctx.gen = ws_obj.generation if use_ws else None
        ctx.save_for_backward(*params)
        ctx.out_rows = out_rows
        C = dims[-1]
        if eval_rows is not None:
            ev = h.index_select(0, eval_rows)[:, :C].contiguous()
        else:
            ev = h.new_zeros(0, C)
        ctx.mark_non_differentiable(ev)
        if out_rows is not None:
            # only the requested rows leave the node, so autograd never holds a dense
            # [V, C] output gradient (a project-first last layer computed just those rows)
            if restrict_last and specs[-1][1] and not specs[-1][0]:
                return (h[:, :C].contiguous() if C != h.shape[1] else h), ev
            return h.index_select(0, out_rows)[:, :C].contiguous(), ev
        return (h[:, :C] if C != h.shape[1] else h), ev

    @staticmethod
    def backward(ctx, gy, _g_eval=None):
        params = ctx.saved_tensors
        graph: DistGraph = ctx.graph
        acts, masks, specs, dims_true = ctx.acts, ctx.masks, ctx.specs, ctx.dims
        dims = ctx.dims_p  # everything below runs at the padded widths
        ctx.acts = ctx.masks = None
        ws_obj, use_ws = ctx.ws, ctx.use_ws
        if use_ws and ws_obj.generation != ctx.gen:
            raise RuntimeError("SAGEStackFn: workspace reused by another forward before "
                               "this backward; run backward before the next forward")
        n = len(specs)
        x0 = acts[0]
        L, dt = x0.shape[0], x0.dtype
        rc, X_ext = ctx.rc, ctx.X_ext
        ctx.X_ext = None
        if rc is not None:
            L = rc.L  # acts[0] holds the L1 extended first-layer rows
        L1 = rc.L1 if rc is not None else L
        V = (lambda name, F: ws_obj.view(name, L, F)) if use_ws else \
            (lambda name, F: torch.empty(L, F, dtype=dt, device=x0.device))
        V1 = (lambda name, F: ws_obj.view(name, L1, F)) if use_ws else \
            (lambda name, F: torch.empty(L1, F, dtype=dt, device=x0.device))
        C, Cp = dims_true[-1], dims[-1]
        gyp = gy.to(dt)
        if Cp != C:
            gyp = Fn.pad(gyp, (0, Cp - C))
        # Output-layer gradient sparsity: dL/dy is zero off the loss rows, so a
        # project-first last layer (y = A z + h Ws, z = h Wn) back-propagates through
        # A[rows, :]^T only, and its g-side GEMMs run on |rows| rows (exact, not an
        # approximation: the dense path would multiply by zero rows).
        lr, lpf = specs[n - 1]
        sparse_last = ctx.out_rows is not None and lpf and not lr
        if sparse_last:
            g = gyp.contiguous()
        elif ctx.out_rows is not None:
            g = V("tmp_a", Cp)
            g.zero_()
            g.index_copy_(0, ctx.out_rows, gyp)
        else:
            g = gyp.contiguous()
            if g is gy:
                g = g.clone()  # never modify the caller's gradient in place
        grads = [None] * len(params)
        dx0 = None
        g_masked = False  # g already carries this layer's ReLU derivative (fused epilogue)
        for i in reversed(range(n)):
            relu, pf = specs[i]
            ws, wn, b = params[3 * i], params[3 * i + 1], params[3 * i + 2]
            ws_, wn_, _ = _padded(params, i, dims, dt)
            r_in, r_out = dims_true[i], dims_true[i + 1]
            if i == n - 1 and sparse_last:
                masks[i] = None
                rows = ctx.out_rows
                x = acts[i]
                acts[i] = None
                x_rows = x.index_select(0, rows)
                grads[3 * i] = wgrad(x_rows, g)[:r_in, :r_out].to(ws.dtype)
                if b is not None:
                    grads[3 * i + 2] = col_sum_f32(g)[:r_out].to(b.dtype)
                dz = graph.aggregate_T_rows(g, rows, mean=True, out=V("tmp_b", dims[i + 1]))
                grads[3 * i + 1] = wgrad(x, dz)[:r_in, :r_out].to(wn.dtype)
                dx = None
                if i > 0 or ctx.x0_requires_grad:
                    prev = masks[i - 1] if i > 0 else None
                    mask_in = prev[1] if isinstance(prev, tuple) else None
                    # dh = mask * (dz Wn^T) + scatter_rows(mask_rows * (g Ws^T)); a
                    # non-fused mask is applied to all of dh at the next layer instead
                    if _fusable(dz, dims[i], dims[i + 1]):
                        dx = dual_gemm(dz, wn_, out=x if i > 0 else None, mask_in=mask_in)
                    elif mask_in is not None:
                        raise RuntimeError("SAGEStackFn: tile32 ReLU mask needs the fused "
                                           "input-gradient GEMM")
                    else:
                        dx = torch.mm(dz, wn_.t(), out=x) if i > 0 else dz @ wn_.t()
                    p = g @ ws_.t()
                    if mask_in is not None:
                        p = p * (x_rows > 0)
                    dx.index_add_(0, rows, p)
                    g_masked = mask_in is not None
                    del p
                del dz, x, x_rows
                g = dx
                if i == 0:
                    dx0 = dx
                continue
            m = masks[i]
            masks[i] = None
            if relu:
                if isinstance(m, tuple):
                    if not g_masked:
                        raise RuntimeError("SAGEStackFn: tile32 ReLU mask was not consumed by "
                                           "the fused input-gradient GEMM")
                elif m.dtype == torch.int32:
                    K.relu_mask_bwd(g, m)
                else:
                    g = torch.where(m > 0, g, torch.zeros((), dtype=g.dtype, device=g.device))
            del m
            x = acts[i]
            acts[i] = None
            recyclable = i > 0  # hidden activations are private to this node
            need_dx = i > 0 or ctx.x0_requires_grad
            # the previous layer's mask, applied inside the fused dx GEMM when it is tile32
            prev = masks[i - 1] if i > 0 else None
            fuse_dx = _bwd_fused(specs, dims, i, need_dx, g)
            mask_in = prev[1] if (fuse_dx and isinstance(prev, tuple)) else None
            g_masked = mask_in is not None

            ext1 = rc is not None and i == 1  # x has the L1 extended rows, g the owned L
            xs = x[:L] if ext1 else x
            # below a loss-row-sparse output layer, g is zero off the loss rows and their
            # neighbours: the transposed aggregation walks only those sources (exact)
            sup = graph.grad_support(ctx.out_rows) if (sparse_last and i == n - 2) \
                else None

            # bias gradient (column sums of g) formed by aggregate_T's pre-scale pass
            gsum = [] if b is not None else None

            def self_grads(i=i, x=xs, g=g, ws=ws, b=b, r_in=r_in, r_out=r_out, gsum=gsum):
                # W_self / bias gradients need no aggregation: on a multi-GPU graph they
                # run while the layer's reverse halo exchange is on the links
                grads[3 * i] = wgrad(x, g)[:r_in, :r_out].to(ws.dtype)
                if b is not None:
                    cs = gsum[0] if gsum else col_sum_f32(g)
                    grads[3 * i + 2] = cs[:r_out].to(b.dtype)

            dx = None
            if pf:
                dz = graph.aggregate_T(g, mean=True, out=V("tmp_b", dims[i + 1]),
                                       overlap=self_grads, support=sup)
                grads[3 * i + 1] = wgrad(x, dz)[:r_in, :r_out].to(wn.dtype)
                if need_dx:
                    if fuse_dx:
                        dx = dual_gemm(g, ws_, dz, wn_, out=x if recyclable else None,
                                       mask_in=mask_in)
                    else:
                        dx = torch.mm(g, ws_.t(), out=x) if recyclable else g @ ws_.t()
                        dx.addmm_(dz, wn_.t())
                del dz
            elif ext1:
                # halo recomputation: u = A^T g over the owned AND halo rows of h1 (the
                # halo part stays here instead of going to the owners), then
                #   dW_neigh = h1_ext^T u,  dh1[own] = g Ws^T + u[own] Wn^T,
                #   dh1[halo] = u[halo] Wn^T   (masked by layer 0's ReLU bits)
                Lp = rc.Lp
                F2 = dims[i + 1]
                u = V1("tmp_a", F2)
                if Lp > L:
                    u[L:Lp].zero_()
                scratch = ws_obj.slots["tmp_b"] if use_ws else None
                graph.aggregate_T(g, mean=True, out=u[:L], scratch=scratch,
                                  overlap=self_grads, halo_out=u[Lp:L1], colsum=gsum,
                                  support=sup)
                del scratch
                grads[3 * i + 1] = wgrad(x, u)[:r_in, :r_out].to(wn.dtype)
                if fuse_dx:
                    # the L1-row tile32 mask: owned rows are its first tiles, the halo rows
                    # start at tile Lp / 32 (Lp is a multiple of the 256-row mask group)
                    w_own = tile32_mask_words(L, dims[i])
                    w0, wh = tile32_mask_words(Lp, dims[i]), tile32_mask_words(L1 - Lp, dims[i])
                    dual_gemm(g, ws_, u[:L], wn_, out=x[:L],
                              mask_in=None if mask_in is None else mask_in[:w_own])
                    dual_gemm(u[Lp:L1], wn_, out=x[Lp:L1],
                              mask_in=None if mask_in is None else mask_in[w0:w0 + wh])
                else:
                    torch.mm(g, ws_.t(), out=x[:L])
                    x[:L].addmm_(u[:L], wn_.t())
                    torch.mm(u[Lp:L1], wn_.t(), out=x[Lp:L1])
                if Lp > L:
                    x[L:Lp].zero_()
                dx = x
                del u
            elif need_dx and dims[i + 1] <= 2 * dims[i]:
                # u = A^T g gives both gradients with ONE SpMM at F_out:
                #   dW_neigh = (A h)^T g = h^T u,   dh = g W_self^T + u W_neigh^T
                # (instead of recomputing A h AND aggregating A^T (g W_neigh^T))
                u_name = "tmp_b" if (i == n - 1 and ctx.out_rows is not None) else "tmp_a"
                # the other temp slot is free here: pre-scaled (unweighted) SpMM passes
                scratch = ws_obj.slots["tmp_b" if u_name == "tmp_a" else "tmp_a"] \
                    if use_ws and i < n - 1 else None
                u = graph.aggregate_T(g, mean=True, out=V(u_name, dims[i + 1]),
                                      scratch=scratch, overlap=self_grads, colsum=gsum,
                                      support=sup)
                del scratch
                grads[3 * i + 1] = wgrad(x, u)[:r_in, :r_out].to(wn.dtype)
                if fuse_dx:
                    # W_self / W_neigh as stored ([F_in, F_out]) are the transposed right
                    # operands of g W^T: no weight copy
                    dx = dual_gemm(g, ws_, u, wn_, out=x if recyclable else None,
                                   mask_in=mask_in)
                else:
                    dx = torch.mm(g, ws_.t(), out=x) if recyclable else g @ ws_.t()
                    dx.addmm_(u, wn_.t())
                del u
            else:
                self_grads()
                # tmp_a may still hold g for the last layer: recompute into tmp_b then
                a_name = "tmp_b" if (i == n - 1 and ctx.out_rows is not None) else "tmp_a"
                V0 = V1 if (rc is not None and i == 0) else V
                if i == 0 and ctx.keep0:
                    a_buf = a = V0("agg0", dims[0])  # kept by forward: no recompute
                elif i == n - 1 and ctx.out_rows is not None and dims[i] > dims[-1]:
                    a_buf = torch.empty(L, dims[i], dtype=dt, device=x.device)
                else:
                    a_buf = V0(a_name, dims[i])
                if not (i == 0 and ctx.keep0):
                    if rc is not None and i == 0:
                        a = rc.aggregate0(X_ext, a_buf)
                    else:
                        a = graph.aggregate(x, mean=True, out=a_buf,
                                            static=i == 0 and not ctx.x0_requires_grad)
                grads[3 * i + 1] = wgrad(a, g)[:r_in, :r_out].to(wn.dtype)
                if need_dx:
                    t = torch.mm(g, wn_.t(), out=a)
                    dx = graph.aggregate_T(t, mean=True, out=x if recyclable else None,
                                           support=sup)
                    del t
                    dx.addmm_(g, ws_.t())
                del a, a_buf
            del x
            g = dx
            if i == 0:
                dx0 = dx
        return (dx0, None, None, None, None, None, None, *grads)


class GraphSAGE(nn.Module):
    """``num_layers`` SAGE-mean layers (ReLU between, none after the last) -> logits.

    With ``dropout == 0`` the forward runs as one :class:`SAGEStackFn` node (buffer
    recycling, bit masks); otherwise as per-layer :class:`SAGEConv` nodes.
    """

    def __init__(self, in_dim: int, hidden: int, out_dim: int, num_layers: int = 3,
                 dropout: float = 0.0, save_agg: Optional[bool] = None):
        super().__init__()
        dims = [in_dim] + [hidden] * (num_layers - 1) + [out_dim]
        self.layers = nn.ModuleList(
            SAGEConv(dims[i], dims[i + 1], relu=(i < num_layers - 1), save_agg=save_agg)
            for i in range(num_layers)
        )
        self.dropout = dropout
        self._workspace = SageWorkspace()

    def forward(self, x: torch.Tensor, graph: DistGraph,
                out_rows: Optional[torch.Tensor] = None,
                eval_rows: Optional[torch.Tensor] = None,
                restrict_last: bool = False):
        """Logits for all local vertices, or only for ``out_rows`` (e.g. the train split:
        the full last layer is still computed, but no dense [V, C] gradient is held).

        With ``eval_rows`` the call returns ``(logits, eval_logits)``: the logits of the
        validation/test vertices from the same full-graph forward (no gradient).
        ``restrict_last=True`` aggregates only ``out_rows`` in a project-first output layer
        (train-rows-only step; not a full-graph forward, see :class:`SAGEStackFn`)."""
        if self.dropout == 0 or not self.training:
            specs = tuple((l.relu, l.project_first()) for l in self.layers)
            params = []
            for l in self.layers:
                params += [l.w_self, l.w_neigh, l.bias]
            ws = self._workspace if (self.training and torch.is_grad_enabled()) else None
            out, ev = SAGEStackFn.apply(x, graph, specs, out_rows, ws,
                                        bool(restrict_last and out_rows is not None),
                                        eval_rows, *params)
            return out if eval_rows is None else (out, ev)
        for i, layer in enumerate(self.layers):
            x = layer(x, graph)
            if self.dropout > 0 and self.training and i < len(self.layers) - 1:
                x = Fn.dropout(x, self.dropout, training=True)
        out = x if out_rows is None else x.index_select(0, out_rows)
        if eval_rows is None:
            return out
        return out, x.index_select(0, eval_rows).detach()

    def num_message_edges(self, graph: DistGraph) -> int:
        """Directed message edges aggregated per layer on this rank (``E_msg``)."""
        n = graph.interior.nnz
        if graph.halo is not None:
            n += graph.halo.nnz
        return n
