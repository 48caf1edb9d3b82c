"""Dense helpers for tall-skinny GNN shapes (rows = vertices, up to 10^8).

* :func:`wgrad` — weight gradient ``x^T g`` ([L,K]^T [L,N], L ~ 1e8, K,N <= 256) with an
  fp32 result. A plain GEMM call gives hipBLASLt a 256x256 output = 16 tiles for 256 CUs
  (79 ms per call on MI355X at L = 111M, profiles/); here the rows are cut into chunks
  and run as one batched GEMM (split-K over the batch), then the fp32 partial products
  are summed (deterministic, fixed order).
* :func:`col_sum_f32` — bias gradient via the native column-sum kernel.
* :func:`deferred_wgrad` — weight gradients of the library's linears computed on a side
  stream, off the backward's critical path.
"""
from __future__ import annotations

import contextlib
from typing import Callable, Optional, Sequence

import torch

from . import f32 as F32
from . import kernels as K


def mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b`` with an fp32 result (bf16 operands, fp32 accumulate)."""
    if a.is_cuda and a.dtype != torch.float32:
        try:
            return torch.mm(a, b, out_dtype=torch.float32)
        except (RuntimeError, TypeError):
            pass
    return torch.mm(a, b).float()


_PARTIALS: dict = {}


def _partials(dev: torch.device, n: int) -> torch.Tensor:
    """Resident fp32 workspace for the split-K partial products, grown on demand and kept:
    allocating ~2 GB per call next to a 269 GB working set made the caching allocator
    free and re-map blocks (184 ms of host time per wgrad, profiles/). Keyed by (device,
    current stream): a wgrad issued on a side stream gets its own buffer, so two streams
    never race on one workspace. :func:`release_workspace` frees them."""
    key = (dev, torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0)
    buf = _PARTIALS.get(key)
    if buf is None or buf.numel() < n:
        # drop the old buffer BEFORE allocating the larger one (peak = new, not old + new)
        buf = None
        _PARTIALS.pop(key, None)
        buf = torch.empty(n, dtype=torch.float32, device=dev)
        _PARTIALS[key] = buf
    return buf[:n]


def release_workspace() -> None:
    """Free the resident split-K workspaces (e.g. before a memory-hungry phase)."""
    _PARTIALS.clear()


# ------------------------------------------------------------- deferred weight gradients
class _Deferral:  # process-wide: the autograd engine runs GPU backward on its own thread
    active = False
    calls = 0  # backward calls whose parameter gradients went to the side stream
    pending: dict = {}  # id(leaf) -> [leaf, buffer]: this block's side-stream gradients


_DEFER = _Deferral()
_SIDE: dict = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    s = _SIDE.get(dev.index)
    if s is None:
        s = _SIDE[dev.index] = torch.cuda.Stream(dev)
    return s


@contextlib.contextmanager
def deferred_wgrad(enabled: bool = True):
    """Inside the block, the backward of :func:`linear`, :func:`linear_sum` and
    ``ops.act.linear_act`` computes each weight (and bias) gradient on ONE side stream
    into a per-parameter buffer, while the data-gradient chain goes on on the current
    stream. Leaving the block joins the side stream into the current one and adds each
    buffer into the parameter's ``.grad`` there (or makes it the ``.grad``), so the
    gradients are complete for what follows (gradient sync, optimizer). ``.grad`` itself is
    only ever touched on the current stream: a parameter whose gradient also arrives
    through autograd's own accumulation (another op, a non-slice view) stays correct.

    For steps of many small kernels (GraphCast's MLPs at 10^5 rows per rank, where one
    GEMM fills a fraction of the 256 CUs) the weight gradients then run in the data
    chain's idle CUs instead of after each of its kernels. A buffer sums its terms in the
    backward's issue order, so a parameter whose every gradient is deferred gets exactly
    the inline result (bitwise). For ``.backward()``: the deferred inputs get no gradient
    through autograd (``torch.autograd.grad`` would not see them). Capturable (the side
    stream forks from and joins the capturing stream)."""
    if not enabled or not torch.cuda.is_available():
        yield
        return
    prev, prev_pending = _DEFER.active, _DEFER.pending
    _DEFER.active, _DEFER.pending = True, {}
    cur = torch.cuda.current_stream()
    try:
        yield
    finally:
        pending = _DEFER.pending
        _DEFER.active, _DEFER.pending = prev, prev_pending
        s = _SIDE.get(cur.device.index)
        if s is not None:
            cur.wait_stream(s)
        for leaf, buf in pending.values():
            buf.record_stream(cur)  # (made on the side stream, read and freed here)
            if leaf.grad is None:
                leaf.grad = buf
            else:
                leaf.grad.add_(buf)


def _leaf_target(p: torch.Tensor):
    """(leaf parameter, (size, stride, offset) of ``p`` inside it, or None for the leaf
    itself) or None when ``p`` is neither a leaf nor a slice of a contiguous one."""
    if not p.requires_grad:
        return None
    b = p if p.is_leaf else p._base
    if b is None or not b.is_leaf or not b.requires_grad or not b.is_contiguous():
        return None
    if b is p:
        return p, None
    return b, (p.size(), p.stride(), p.storage_offset() - b.storage_offset())


def defer_param_grads(params: Sequence[torch.Tensor], compute: Callable[[], Sequence],
                      keep_alive: Sequence[torch.Tensor] = ()) -> bool:
    """Under :func:`deferred_wgrad`: run ``compute()`` (returning one gradient per entry
    of ``params``) on the side stream and add each into its parameter's block buffer;
    returns True (the caller then returns None for those inputs). False, with nothing
    run, when deferral is off or a parameter is not a plain leaf / slice of one.
    ``keep_alive``: tensors ``compute`` reads (their memory is held for the side stream)."""
    if not _DEFER.active or not params or not params[0].is_cuda:
        return False
    targets = [_leaf_target(p) for p in params]
    if any(t is None for t in targets):
        return False
    cur = torch.cuda.current_stream()
    side = _side_stream(params[0].device)
    pend = _DEFER.pending
    slots = []  # per target: (pending entry, view) — entry [leaf, None] until first write
    for leaf, view in targets:
        e = pend.get(id(leaf))
        if e is None:
            e = pend[id(leaf)] = [leaf, None]
        if e[1] is None and view is not None:
            e[1] = torch.zeros_like(leaf)  # on the current stream, before the fork
        slots.append((e, view))
    _DEFER.calls += 1
    side.wait_stream(cur)
    for t in keep_alive:
        t.record_stream(side)
    with torch.cuda.stream(side):
        for (e, view), o in zip(slots, compute()):
            buf = e[1]
            if buf is None:  # the parameter's first term: it becomes the buffer
                e[1] = o.to(e[0].dtype).contiguous()
            elif view is None:
                buf.add_(o.to(buf.dtype))
            else:
                buf.as_strided(view[0], view[1], buf.storage_offset() + view[2]).add_(
                    o.to(buf.dtype))
    return True


def _bmm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if a.is_cuda and a.dtype != torch.float32:
        out = _partials(a.device, a.shape[0] * a.shape[1] * b.shape[2]).view(
            a.shape[0], a.shape[1], b.shape[2])
        try:
            return torch.bmm(a, b, out_dtype=torch.float32, out=out)
        except (RuntimeError, TypeError):
            pass
        try:
            return torch.bmm(a, b, out_dtype=torch.float32)
        except (RuntimeError, TypeError):
            pass
    return torch.bmm(a, b).float()


def _wgrad_rows_per_chunk(L: int, K: int, N: int, budget: int = 2 << 30) -> int:
    """Chunk rows for the split-K batch: small chunks (many independent [K, N] products)
    measured fastest on MI355X at L = 111M (K = N = 256: 2^14 rows 20.6 ms, 2^16 27.2 ms,
    2^18 30.0 ms; benchmarks/bench_wgrad.py), bounded so the fp32 partials stay under
    ``budget`` bytes."""
    c = 1 << 14
    while (L // c) * K * N * 4 > budget:
        c *= 2
    return c


def wgrad(x: torch.Tensor, g: torch.Tensor, rows_per_chunk: int = 0) -> torch.Tensor:
    """``x^T @ g`` in fp32 for tall ``x [L, K]``, ``g [L, N]`` (row-contiguous).
    ``rows_per_chunk`` 0 = size-aware default. The wider operand goes first (the library
    kernel it selects streams that operand once: K=128, N=256 19.3 ms -> ~14.6 ms)."""
    L = x.shape[0]
    if L == 0:
        return torch.zeros(x.shape[1], g.shape[1], dtype=torch.float32, device=x.device)
    if x.is_cuda and x.shape[1] < g.shape[1]:
        return wgrad(g, x, rows_per_chunk).t()
    if rows_per_chunk <= 0:
        rows_per_chunk = _wgrad_rows_per_chunk(L, x.shape[1], g.shape[1])
    nb = L // rows_per_chunk
    if not x.is_cuda or nb < 2 or not (x.is_contiguous() and g.is_contiguous()):
        return mm_f32(x.t(), g)
    Lm = nb * rows_per_chunk
    xb = x[:Lm].view(nb, rows_per_chunk, x.shape[1]).transpose(1, 2)
    gb = g[:Lm].view(nb, rows_per_chunk, g.shape[1])
    out = _bmm_f32(xb, gb).sum(0)
    if Lm < L:
        out += mm_f32(x[Lm:].t(), g[Lm:])
    return out


def col_sum_f32(g: torch.Tensor) -> torch.Tensor:
    """fp32 column sums without an fp32 copy of ``g``."""
    return K.col_sum(g)


def _wgrad_chunk(L: int) -> int:
    return 0 if L >= 1 << 23 else _auto_rows_per_chunk(L)


def _auto_rows_per_chunk(L: int) -> int:
    """Chunk so the batched wgrad has >= ~128 independent output tiles (256 CUs), but
    keeps chunks >= 4096 rows."""
    c = 4096
    while L // c > 128:
        c *= 2
    return c


class _LinearFn(torch.autograd.Function):
    """``y = x W^T + b`` whose backward computes dW with the split-K batched GEMM and
    db with the native column sum (the library GEMM for a 128x128 weight gradient over
    10^6 rows runs on 2 workgroups; profiles/graphcast_1gpu_kernel_stats.txt)."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        ctx.b = b  # the parameter itself (deferred_wgrad adds into its .grad)
        if x.dim() == 2:  # fp32 on the GPU: the exact-f32 MFMA GEMM, bias fused
            return F32.linear_fwd(x, W, b)
        return torch.nn.functional.linear(x, W, b)

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        N = W.shape[0]
        g2 = g.reshape(-1, N).contiguous()
        x2 = x.reshape(-1, W.shape[1])
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            dx = F32.linear_dgrad([g2], [W]).reshape(x.shape)
        want_b = ctx.has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] and g2.is_cuda and _DEFER.active:
            ps = [W, ctx.b] if want_b else [W]

            def comp():
                r = F32.linear_wgrad(g2, x2, W, bias=want_b)
                if r is None:
                    r = wgrad(g2, x2.contiguous(), _wgrad_chunk(g2.shape[0]))
                    r = (r, col_sum_f32(g2)) if want_b else r
                return r if isinstance(r, tuple) else (r,)

            if defer_param_grads(ps, comp, keep_alive=(g2, x2)):
                return dx, None, None
        if ctx.needs_input_grad[1]:
            # fp32: split-M MFMA accumulator (and the bias gradient from the same pass)
            dW = F32.linear_wgrad(g2, x2, W, bias=want_b)
            if isinstance(dW, tuple):
                dW, db = dW
                db = db.to(W.dtype)
                want_b = False
            if dW is None and g2.is_cuda:
                # >= 8M rows (R-GCN relation linears): the 2^14-row split-K default
                # (1/8 MAG240M step 378 -> 357 ms); fewer rows (GraphCast, 1-2M): >= 4096
                # rows x <= 128 chunks (50.5 -> 46.4 ms)
                dW = wgrad(g2, x2.contiguous(), _wgrad_chunk(g2.shape[0]))
            elif dW is None:
                dW = g2.t().to(torch.float64 if g2.dtype == torch.float64 else torch.float32) @ \
                    x2.to(torch.float64 if g2.dtype == torch.float64 else torch.float32)
            dW = dW.to(W.dtype)
        if want_b:
            db = (col_sum_f32(g2) if g2.is_cuda else g2.sum(0)).to(W.dtype)
        return dx, dW, db


def linear(x: torch.Tensor, W: torch.Tensor, b=None) -> torch.Tensor:
    """Drop-in for ``F.linear`` with a tall-skinny-aware backward."""
    if torch.is_autocast_enabled() and x.is_cuda:
        dt = torch.get_autocast_dtype("cuda")
        x, W = x.to(dt), W.to(dt)
        b = None if b is None else b.to(dt)
    return _LinearFn.apply(x, W, b)


def tile32_mask_words(M: int, N: int) -> int:
    """int64 words of a dual-GEMM keep mask for an [M, N] output."""
    return (M + 255) // 256 * 8 * (N // 32) * 16


def dual_gemm_supported(A1: torch.Tensor, N: int, K2: int = 0) -> bool:
    ks = (128, 192, 256)
    return (A1.is_cuda and A1.dtype == torch.bfloat16 and N in ks and A1.shape[1] in ks
            and (K2 == 0 or K2 in ks) and A1.stride(1) == 1 and A1.stride(0) % 8 == 0)


def dual_gemm(A1: torch.Tensor, B1t: torch.Tensor, A2=None, B2t=None, bias=None, cin=None,
              out=None, relu: bool = False, mask_out=None, mask_in=None) -> torch.Tensor:
    """``out = epi(A1 B1 (+ A2 B2) (+ bias) (+ cin))`` on the native MFMA kernel
    (csrc/kernels/dual_gemm.hip); ``B*t`` are the transposed right operands ``[N, K]``."""
    from .. import _native

    if out is None:
        out = torch.empty(A1.shape[0], B1t.shape[0], dtype=A1.dtype, device=A1.device)
    b = None if bias is None else bias.float().contiguous()
    _native.ops().dual_gemm(A1, B1t.contiguous(), A2,
                            None if B2t is None else B2t.contiguous(), b, cin, out, mask_out,
                            mask_in, bool(relu))
    return out


def dual_gemm_shape_ok(N: int, K1: int, K2: int = 0) -> bool:
    ks = (128, 192, 256)
    return N in ks and K1 in ks and (K2 == 0 or K2 in ks)


def _native_linear_sum_ok(xs, Ws, acc) -> bool:
    N = Ws[0].shape[0]
    if not (xs[0].is_cuda and all(x.dtype == torch.bfloat16 for x in xs)):
        return False
    if acc is not None and (acc.dtype != torch.bfloat16 or not acc.is_contiguous()
                            or acc.shape != (xs[0].shape[0], N)):
        return False
    return all(x.dim() == 2 and x.is_contiguous() and W.shape[0] == N
               and dual_gemm_shape_ok(N, x.shape[1]) for x, W in zip(xs, Ws))


class _LinearSumFn(torch.autograd.Function):
    """``y = sum_i x_i W_i^T + b (+ acc)`` (R-GCN: skip + one linear per relation into the
    same destination). On the GPU the terms go through the native MFMA dual GEMM two at a
    time, chaining the running sum through its ``cin`` input, so the per-term outputs and
    the elementwise adds never touch HBM; backward: ``dx_i = g W_i`` on the same kernel,
    split-K ``dW_i``, native column-sum ``db``, ``dacc = g``."""

    @staticmethod
    def forward(ctx, b, acc, *flat):
        xs, Ws = list(flat[0::2]), list(flat[1::2])
        ctx.save_for_backward(*flat)
        ctx.has_b, ctx.has_acc = b is not None, acc is not None
        ctx.native = _native_linear_sum_ok(xs, Ws, acc)
        if ctx.native:
            out = torch.empty(xs[0].shape[0], Ws[0].shape[0], dtype=xs[0].dtype,
                              device=xs[0].device)
            cin = acc
            for k in range(0, len(xs), 2):
                two = k + 1 < len(xs)
                dual_gemm(xs[k], Ws[k].to(xs[k].dtype), xs[k + 1] if two else None,
                          Ws[k + 1].to(xs[k].dtype) if two else None,
                          bias=b if k == 0 else None, cin=cin, out=out)
                cin = out
            return out
        if xs[0].is_cuda and xs[0].dtype == torch.float32 and F32.LINEAR_ON and all(
                x.dim() == 2 and x.stride(1) == 1 and x.shape[1] % 32 == 0 for x in xs) \
                and F32.tileable(Ws[0].shape[0]):
            # fp32: the exact-f32 MFMA GEMM two terms per call, the running sum (and acc)
            # chained through cin
            out = None
            cin = acc
            for k in range(0, len(xs), 2):
                two = k + 1 < len(xs)
                out = F32.gemm_f32(xs[k], Ws[k].t().contiguous(), xs[k + 1] if two else None,
                                   Ws[k + 1].t().contiguous() if two else None,
                                   bias=b if k == 0 else None, cin=cin, out=out)
                cin = out
            return out
        out = torch.nn.functional.linear(xs[0], Ws[0], b)
        for x, W in zip(xs[1:], Ws[1:]):
            out = out + torch.nn.functional.linear(x, W)
        return out if acc is None else out + acc

    @staticmethod
    def backward(ctx, g):
        flat = ctx.saved_tensors
        xs, Ws = flat[0::2], flat[1::2]
        g = g.contiguous()
        grads = []
        wi = [i for i in range(len(Ws)) if ctx.needs_input_grad[3 + 2 * i]]
        deferred = g.is_cuda and _DEFER.active and bool(wi)
        for i, (x, W) in enumerate(zip(xs, Ws)):
            dx = dW = None
            if ctx.needs_input_grad[2 + 2 * i]:
                if ctx.native and dual_gemm_shape_ok(x.shape[1], W.shape[0]):
                    dx = dual_gemm(g, W.to(g.dtype).t().contiguous())
                else:
                    dx = F32.linear_dgrad([g], [W])
            if ctx.needs_input_grad[3 + 2 * i] and not deferred:
                dW = F32.linear_wgrad(g, x, W)  # fp32: split-M MFMA accumulator
                if dW is None and g.is_cuda:
                    L = g.shape[0]
                    dW = wgrad(g, x, 0 if L >= 1 << 23 else _auto_rows_per_chunk(L))
                elif dW is None:
                    adt = torch.float64 if g.dtype == torch.float64 else torch.float32
                    dW = g.t().to(adt) @ x.to(adt)
                dW = dW.to(W.dtype)
            grads += [dx, dW]
        db = None
        if deferred:
            ps = [Ws[i] for i in wi]

            def comp():
                out = []
                for i in wi:
                    r = F32.linear_wgrad(g, xs[i], Ws[i])
                    out.append(r if r is not None else
                               wgrad(g, xs[i].contiguous(), _wgrad_chunk(g.shape[0])))
                return out

            if not defer_param_grads(ps, comp, keep_alive=(g, *[xs[i] for i in wi])):
                for i in wi:  # not deferrable (a parameter behind another view)
                    r = F32.linear_wgrad(g, xs[i], Ws[i])
                    r = r if r is not None else wgrad(g, xs[i].contiguous(),
                                                      _wgrad_chunk(g.shape[0]))
                    grads[2 * i + 1] = r.to(Ws[i].dtype)
        if ctx.has_b and ctx.needs_input_grad[0]:
            db = col_sum_f32(g) if g.is_cuda else \
                g.to(torch.float64 if g.dtype == torch.float64 else torch.float32).sum(0)
        dacc = g if ctx.has_acc and ctx.needs_input_grad[1] else None
        return (db, dacc, *grads)


def linear_sum(terms, b=None, acc=None) -> torch.Tensor:
    """``sum_i x_i W_i^T + b (+ acc)`` for ``terms = [(x_i, W_i), ...]`` (see
    :class:`_LinearSumFn`)."""
    xs = [x for x, _ in terms]
    Ws = [W for _, W in terms]
    if torch.is_autocast_enabled() and xs[0].is_cuda:
        dt = torch.get_autocast_dtype("cuda")
        xs = [x.to(dt) for x in xs]
        Ws = [W.to(dt) for W in Ws]
        b = None if b is None else b.to(dt)
        acc = None if acc is None else acc.to(dt)
    flat = [t for pair in zip(xs, Ws) for t in pair]
    out = _LinearSumFn.apply(b, acc, *flat)
    return out
