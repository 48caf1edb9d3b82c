"""Memory-lean fp32 full-graph GraphSAGE step (the headline config at the reference's
precision).

The reference trains in fp32 only (DGraph/distributed/csrc/torch_local_kernels.cu:43-46;
experiments/OGB/main.py:129-184 run the full-graph epoch: forward of every vertex, masked
loss, backward, optimizer step). At the ogbn-papers100M shape a plain fp32 layer-by-layer
autograd step needs ~420 GB on one GPU (features 57 GB, two hidden activations 114 GB each,
their aggregates and gradients as large). This executor is a hand-scheduled forward and
backward over ROW CHUNKS that never materialises an aggregate, a logit matrix or a dense
hidden gradient:

forward (per row chunk c, interior + halo parts, every vertex of every layer):
  F0  a_c = mean_N(x)_c            -> h1[c] = relu([x_c | a_c] [Ws0; Wn0] + b0)
  F1  a_c = mean_N(h1)_c           -> h2[c] = relu([h1_c | a_c] [Ws1; Wn1] + b1)
  F2  a_c = mean_N(h2)_c           -> z_c = [h2_c | a_c] [Ws2; Wn2] + b2 (all rows' logits)
      loss rows of c: cross-entropy, dz (kept, |T| rows), dW2 += [h2 | a]_T^T dz;
      validation/test rows of c: argmax hits.          (aggregate-first everywhere)
backward, with S = T + N(T) (+ rows remote loss rows reach: the gradient support):
  B2  dZ1[S] = keep(h2 > 0) * (A_T^T (dz Wn2^T / deg_T) + scatter_T(dz Ws2^T))
  B1a over S chunks: dW1 += [h1 | mean_N(h1)]_S^T dZ1      (aggregate of S rows only)
      u1 = (dZ1 Wn1^T) / deg_S
  B1b over row chunks c: dZ0_c = keep(h1_c > 0) * (A^T u1 (column-mapped onto S) +
      scatter_S(dZ1 Ws1^T))_c ;  dW0 += [x_c | mean_N(x)_c]^T dZ0_c
Exact: every term the dense backward has is computed (the omitted products are with rows
that are zero by construction). Live device memory at the papers100M shape, W=1: x 57 GB +
CSR 14 GB + h1 114 GB + h2 114 GB + ~4 GB of chunk buffers; dZ1 and u1 live in h2's
storage after its last use. Kernels: fp32 row-group SpMM with row lists / column maps /
gates (csrc/kernels/spmm_f32.hip), MFMA f32 dual GEMM with bias/ReLU/gate/row-scatter
epilogues (gemm_f32.hip), split-M MFMA weight gradients (wgrad_f32.hip), keep bits
(bits.hip). Deterministic: fixed chunking, fixed reduction orders, no atomics.

Vertex-partitioned graphs (W > 1): halo rows of x are exchanged once (static input), of
h1/h2 once per forward — each issued asynchronously as soon as its layer is done and
overlapped with the next layer's interior aggregation of every row (through a whole-layer
aggregate buffer, or in place in the layer's own output buffer when there is no room for
one); B2 sends the loss rows' contributions to remote support rows (restricted sub-plan of
:class:`~dgraph_amd.parallel.dist_graph.DistGraph`), B1b sends the support rows'
contributions to remote vertices (reverse halo exchange, issued before the B1a work so it
overlaps it). The halo rows are part of the memory plan, which raises MemoryError before
allocating when a configuration cannot fit.

Measured choices (profiles/r03/, PERFORMANCE.md): the SpMM column-pass width follows the
graph's locality (64 columns on a windowed graph, full rows on a structureless one); the
column-mapped transposed aggregation compacts each chunk's mapped entries before gathering;
the chunks run on one stream (the two-stream pipeline and the one-kernel fused layer,
DGRAPH_FUSED_PIPELINE / DGRAPH_FUSED_FWD, are correct but not faster: the fp32 GEMM's
register footprint keeps the memory-bound and the MFMA-bound work from co-residing).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch

from .. import _native
from ..ops import f32 as F32
from ..ops import kernels as K
from ..parallel.dist_graph import DistGraph

# rows per chunk of the row-chunked passes (0 = auto from free memory)
CHUNK_ROWS = int(os.environ.get("DGRAPH_FUSED_CHUNK_ROWS", "0"))
# fp32 GEMMs as bf16x3 split-product MFMAs (csrc/kernels/gemm_x3.hip: fp32-accurate, error vs
# fp64 below the exact-f32 MFMA's); 0 = exact-f32 MFMAs (gemm_f32.hip)
GEMM_X3 = os.environ.get("DGRAPH_GEMM_X3", "0") == "1"
# W = 1: each hidden layer as ONE fused kernel (csrc/kernels/sage_fwd_f32.hip: gather waves
# and MFMA waves co-resident on every CU) instead of chunked aggregation + GEMM launches
FUSED_FWD = os.environ.get("DGRAPH_FUSED_FWD", "0") == "1"
# W > 1: overlap each forward halo exchange with the next layer's interior aggregation
OVERLAP_FWD = os.environ.get("DGRAPH_FUSED_OVERLAP", "1") != "0"


def _ranges(n: int, step: int) -> List[Tuple[int, int]]:
    return [(a, min(n, a + step)) for a in range(0, n, step)] or [(0, 0)]


def _pad_to(n: int, m: int) -> int:
    return (n + m - 1) // m * m


class _Pipe:
    """Two-stage chunk pipeline: stage 1 (the memory-bound aggregation of chunk c into
    buffer c % 2) on the current stream, stage 2 (MFMA GEMMs / weight gradients reading that
    buffer) on a side stream, events ordering buffer reuse. OFF by default
    (DGRAPH_FUSED_PIPELINE=1 turns it on): the fp32 GEMM block takes every SIMD's register
    file, so the two kernels do not co-reside and the streams only add ordering overhead
    (benchmarks/bench_overlap_f32.py: 127.9 ms piped vs 122.7 serial per layer at 1/4
    scale; full step 2060 ms piped vs 2051 serial, profiles/r03/). Off = plain sequence."""

    def __init__(self, dev):
        self.cuda = dev.type == "cuda" and os.environ.get("DGRAPH_FUSED_PIPELINE", "0") == "1"
        if self.cuda:
            # DGRAPH_FUSED_SIDE_PRIO=1: the matrix stage's stream at high priority, so when a
            # chunk's GEMM and the next chunk's aggregation become ready together the GEMM's
            # (LDS-heavy, one-per-CU) blocks are placed first and the aggregation fills the
            # registers left over, instead of the other way round
            prio = -1 if os.environ.get("DGRAPH_FUSED_SIDE_PRIO", "0") == "1" else 0
            self.side = torch.cuda.Stream(dev, priority=prio)
            self.ready = [torch.cuda.Event() for _ in range(2)]
            self.free = [torch.cuda.Event() for _ in range(2)]

    def run(self, items, produce, consume):
        if not self.cuda:
            for k, it in enumerate(items):
                consume(it, produce(it, k % 2), k % 2)
            return
        main = torch.cuda.current_stream()
        self.side.wait_stream(main)
        used = [False, False]
        for k, it in enumerate(items):
            b = k % 2
            if used[b]:
                main.wait_event(self.free[b])
            res = produce(it, b)
            self.ready[b].record(main)
            with torch.cuda.stream(self.side):
                self.side.wait_event(self.ready[b])
                consume(it, res, b)
                self.free[b].record(self.side)
            used[b] = True
        main.wait_stream(self.side)


def supported(model, x: torch.Tensor) -> bool:
    """Shapes the fused executor runs (the GraphSAGE of bench.py / the OGB shapes)."""
    layers = list(model.layers)
    if len(layers) not in (2, 3) or getattr(model, "dropout", 0.0) != 0.0:
        return False
    hid = layers[0].out_dim
    d0 = x.shape[1]
    # input widths up to 128 (narrower features are zero-padded to 64 / 128 columns)
    return (x.dtype == torch.float32 and 0 < d0 <= 128
            and hid == 256 and all(l.out_dim == hid for l in layers[:-1])
            and layers[-1].out_dim <= 176)


def _in_width(d0: int) -> int:
    """Input width the kernels run at: the layer-0 GEMM's K (a multiple of 32) and the
    input weight gradient's K = 2 * width (128 or 256)."""
    return 64 if d0 <= 64 else 128


class FusedSAGE:
    """The fp32 training step of a 2- or 3-layer :class:`~dgraph_amd.models.sage.GraphSAGE`
    (mean aggregator, ReLU between layers, no dropout) over a :class:`DistGraph`.

    ``step()`` runs forward + backward, leaves the weight gradients in ``p.grad`` of the
    model's parameters and returns the loss (device scalar, this rank's share of the global
    mean: the sum over this rank's loss rows divided by the GLOBAL train-row count
    ``n_train``, so an all-reduce of the gradients gives the full-batch gradient).
    ``self.correct`` holds (validation hits, test hits) of the same forward."""

    def __init__(self, model, graph: DistGraph, x: torch.Tensor, train_idx: torch.Tensor,
                 y_train: torch.Tensor, eval_idx: torch.Tensor, y_eval: torch.Tensor,
                 eval_is_val: torch.Tensor, n_train: int, chunk_rows: int = 0):
        if not supported(model, x):
            raise ValueError("FusedSAGE: unsupported model/feature shape")
        dev = x.device
        self.dev = dev
        self.d0_in = x.shape[1]
        self.d0 = _in_width(self.d0_in)
        if self.d0 != self.d0_in:
            # zero feature columns: their aggregates are zero, their weight rows get
            # gradients that are dropped (ogbn-products: 100 -> 128)
            xp = torch.zeros(x.shape[0], self.d0, dtype=x.dtype, device=dev)
            xp[:, :self.d0_in] = x
            x = xp
        self.model, self.g, self.x = model, graph, x.contiguous()
        L, H = graph.L, graph.H
        self.L, self.H = L, H
        self.nl = len(model.layers)
        self.hid = model.layers[0].out_dim
        self.C = model.layers[-1].out_dim
        self.x3 = GEMM_X3 and dev.type == "cuda"
        self._x3_cache: dict = {}
        # logit GEMM width (the bf16x3 tile needs a multiple of 64)
        self.Cp = (192 if self.x3 else 176) if self.C > 128 else (128 if self.C > 64 else 64)
        self.Cg = _pad_to(self.C, 32) if self.C > 128 else self.Cp      # dz width (a K dim)
        if self.Cg not in (128, 176, 192, 256):
            self.Cg = 192
        self.inv_n = 1.0 / max(int(n_train), 1)
        # ---- loss / eval rows, sorted (chunk ranges are searchsorted)
        t, tp = torch.sort(train_idx.long())
        self.T, self.yT = t.contiguous(), y_train[tp].contiguous()
        e, ep = torch.sort(eval_idx.long())
        self.E, self.yE = e.contiguous(), y_eval[ep].contiguous()
        self.E_val = eval_is_val[ep].contiguous()
        self.inv_deg = graph.inv_deg
        self.invdegT = self.inv_deg[self.T].contiguous()
        # ---- gradient support S (rows where dZ of the last hidden layer can be nonzero)
        it_t, _, sub = graph._restricted(self.T)  # A[T, :L]^T (rows L, cols |T|), sub-plan
        parts = [self.T, it_t.compact_rows().row_map.long()]
        if sub is not None:
            parts.append(sub[4].long())
        S = torch.unique(torch.cat(parts))
        self.S = S.contiguous()
        self.nS = S.numel()
        smap = torch.full((L,), -1, dtype=torch.int32, device=dev)
        smap[S] = torch.arange(self.nS, dtype=torch.int32, device=dev)
        self.smap = smap
        self.posT = smap[self.T].long().contiguous()
        self.invdegS = self.inv_deg[S].contiguous()
        self.AT_S = it_t.select_rows(S)            # rows S (compact), cols T (compact)
        self.sub = None
        if sub is not None:
            ht_nz, a2a_sub, st = sub[0], sub[1], sub[2]
            stc = st.compact_rows()
            self.sub = (ht_nz, a2a_sub, stc, smap[stc.row_map].long().contiguous())
        # ---- interior / halo structures
        self.it = graph.interior
        self.halo = graph.halo
        self.hcomp = graph.halo.compact_rows() if graph.halo is not None else None
        self.haloT = graph.halo.transpose() if graph.halo is not None else None
        self.send_st = graph.send_map.transpose_csr().compact_rows() \
            if graph.halo is not None else None
        # entries of the S-row aggregation (B1a), counted on the host once
        self.nnz_S = int((self.it.rowptr[S + 1] - self.it.rowptr[S]).sum())
        if self.halo is not None:
            self.nnz_S += int((self.halo.rowptr[S + 1] - self.halo.rowptr[S]).sum())
        # ---- chunking (the planning above left cached temporaries: return them first, and
        # count what the caching allocator still holds unused as free)
        if dev.type == "cuda":
            torch.cuda.empty_cache()
            free = torch.cuda.mem_get_info(dev)[0] + \
                torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
        else:
            free = 64 << 30
        need_h = (self.nl - 1) * L * self.hid * 4
        self.store_sep = 2 * self.nS > L   # dZ and u do not fit in the last hidden buffer
        if self.store_sep:
            need_h += 2 * self.nS * self.hid * 4
        nT = self.T.numel()
        # dz rows, wgrad slabs, (u_out when it cannot live in the last hidden buffer) and
        # allocator / temporary slack; the chunk arena gets the rest
        self.u_sep = 2 * self.nS + nT > L
        other = 4 * nT * self.Cg + 5 * 4 * 256 * 256 * 256 + (3 << 29) + \
            (4 * nT * self.hid if self.u_sep else 0)
        wA, wB = max(self.hid, self.d0), max(self.Cp, self.hid)
        # W > 1: the received halo rows live through the step — the input's (exchanged once,
        # kept), every hidden layer's (the backward reads them) — and each exchange's send
        # rows while it is in flight: planned here, not discovered by the allocator
        H = graph.H if graph.halo is not None else 0
        n_send = graph.send_map.idx.numel() if graph.halo is not None else 0
        self.halo_bytes = 4 * (H * self.d0 + (self.nl - 1) * H * self.hid + n_send * self.hid)
        need_h += self.halo_bytes
        if dev.type == "cuda" and need_h + other + (1 << 28) > free:
            # fail here, before any allocation (and after every collective of the setup), so a
            # caller can skip the configuration on every rank alike instead of dying mid-step
            raise MemoryError(
                f"FusedSAGE: activations {need_h / 2**30:.1f} GiB (halo rows "
                f"{self.halo_bytes / 2**30:.1f}) + workspace {other / 2**30:.1f} GiB exceed the "
                f"{free / 2**30:.1f} GiB free on {dev}")
        # W > 1: a whole-layer aggregate buffer lets the interior aggregation of EVERY row run
        # while the previous layer's halo rows are in flight (the halo part and the GEMMs
        # follow once they land); without room for it the exchange is waited for up front
        self.agg_full = None
        need_full = L * wA * 4
        if graph.halo is not None and OVERLAP_FWD and free - need_h - other - need_full > (
                16 << 30 if dev.type == "cuda" else 0):
            self.agg_full = torch.empty(L, wA, dtype=torch.float32, device=dev)
            other += need_full
        # the fused hidden-layer kernel's per-block aggregate ring (W = 1, int32 columns)
        self.fwd_ring = self.fwd_err = None
        if (FUSED_FWD and dev.type == "cuda" and graph.halo is None
                and self.it.col.dtype == torch.int32 and self.hid == 256):
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            self.fwd_ring = torch.empty(ncu * 2 * 128 * 256, dtype=torch.float32, device=dev)
            self.fwd_err = torch.zeros(1, dtype=torch.int32, device=dev)
            other += self.fwd_ring.numel() * 4
        spare = max(free - need_h - other, 1 << 28)
        self.pipe = _Pipe(dev)
        # chunk buffers: two of each when the two-stream pipeline runs (chunk c+1 is written
        # while chunk c is read), one otherwise — the freed memory goes to larger chunks
        self.nbuf = 2 if self.pipe.cuda else 1
        per_row = 4 * self.nbuf * (wA + wB)  # aggregate + logit/gradient chunk buffers
        cr = chunk_rows or CHUNK_ROWS
        if cr <= 0:
            cr = int(min(max(spare // per_row, 1 << 16), 1 << 21))
        self.cr = max(256, min(int(cr), max(L, 256)))
        self.chunks = _ranges(L, self.cr)
        self.s_chunks = _ranges(self.nS, self.cr)
        ss = lambda v, a: int(torch.searchsorted(v, torch.tensor(a, device=v.device)))  # noqa
        self.ch_T = [(ss(self.T, r0), ss(self.T, r1)) for r0, r1 in self.chunks]
        self.ch_E = [(ss(self.E, r0), ss(self.E, r1)) for r0, r1 in self.chunks]
        self.ch_S = [(ss(self.S, r0), ss(self.S, r1)) for r0, r1 in self.chunks]
        self.ch_Tloc = [(self.T[a:b] - r0).contiguous()
                        for (r0, _), (a, b) in zip(self.chunks, self.ch_T)]
        self.ch_Eloc = [(self.E[a:b] - r0).contiguous()
                        for (r0, _), (a, b) in zip(self.chunks, self.ch_E)]
        self.ch_Sloc = [(self.S[a:b] - r0).contiguous()
                        for (r0, _), (a, b) in zip(self.chunks, self.ch_S)]
        self.ch_halo = [self._halo_range(self.hcomp, r0, r1) for r0, r1 in self.chunks]
        self.ch_send = [self._halo_range(self.send_st, r0, r1) for r0, r1 in self.chunks]
        # ---- persistent buffers (allocated once: no allocation in the steady state)
        f = dict(dtype=torch.float32, device=dev)
        self.h = [torch.empty(L, self.hid, **f) for _ in range(self.nl - 1)]
        if self.store_sep:
            self.dZ = torch.empty(self.nS, self.hid, **f)
            self.u = torch.empty(self.nS, self.hid, **f) if self.nl == 3 else None
        else:
            hl = self.h[-1].view(-1)
            n = self.nS * self.hid
            self.dZ = hl[:n].view(self.nS, self.hid)
            self.u = hl[n:2 * n].view(self.nS, self.hid) if self.nl == 3 else None
        # ONE chunk arena: two of each chunk buffer (chunk c+1's aggregation, a memory-bound
        # SpMM on the producer stream, runs while chunk c's MFMA GEMMs on the consumer
        # stream read the other one) during the row-chunked passes, and the last hidden
        # layer's keep bits (output-layer backward only, when no chunk buffer is live)
        bits_words = self.nS * (self.hid // 32)
        arena_fl = max(self.nbuf * self.cr * (wA + wB), bits_words)
        self.arena = torch.empty(arena_fl, **f)
        o = 0
        self.bufA2, self.bufB2 = [], []
        for w, lst in ((wA, self.bufA2), (wB, self.bufB2)):
            for _ in range(self.nbuf):
                lst.append(self.arena[o:o + self.cr * w].view(self.cr, w))
                o += self.cr * w
            if self.nbuf == 1:  # index k % 2 reaches the single buffer either way
                lst.append(lst[0])
        self.bufA, self.bufB = self.bufA2[0], self.bufB2[0]
        self.bits = self.arena[:bits_words].view(torch.int32).view(self.nS, self.hid // 32)
        self.dz = torch.zeros(self.T.numel(), self.Cg, **f)  # output-layer gradient rows
        # the output layer's projected gradient rows (B2 only): the last hidden buffer's tail,
        # past dZ and u, is free by then
        if self.u_sep:
            self.u_out = torch.empty(nT, self.hid, **f)
        else:
            tail = self.h[-1].view(-1)[2 * self.nS * self.hid:]
            self.u_out = tail[:nT * self.hid].view(nT, self.hid)
        self.v_self = None
        if self.nl == 3:
            n_used = (2 * self.nS + (0 if self.u_sep else nT)) * self.hid
            if not self.store_sep and n_used + self.nS * self.hid <= L * self.hid:
                self.v_self = self.h[-1].view(-1)[n_used:n_used + self.nS * self.hid].view(
                    self.nS, self.hid)
            elif dev.type != "cuda" or free - need_h > (4 * self.nS * self.hid + (8 << 30)):
                self.v_self = torch.empty(self.nS, self.hid, **f)
            # else: no room — the self term runs as a row-scattered GEMM per chunk
        self.acc_out_s = F32.WgradAcc(self.hid, self.Cg, dev, x3=self.x3)
        self.acc_out_n = F32.WgradAcc(self.hid, self.Cg, dev, x3=self.x3)
        kh = self.hid if self.nl == 3 else self.d0
        self.acc_hid_s = F32.WgradAcc(kh, self.hid, dev, x3=self.x3)
        self.acc_hid_n = F32.WgradAcc(kh, self.hid, dev, x3=self.x3)
        self.acc_in = F32.WgradAcc(2 * self.d0, self.hid, dev, x3=self.x3) if self.nl == 3 else None
        self.row_loss = torch.zeros(nT, **f)
        self.hit = torch.zeros(self.E.numel(), dtype=torch.uint8, device=dev)
        self.E_val_l = self.E_val.long()
        self.correct = torch.zeros(2, dtype=torch.long, device=dev)
        self.record = False
        self._events: list = []
        self._tune_passes()

    # ------------------------------------------------------------------ regions
    def _mark(self, name: str):
        """Record a stream event opening region ``name`` (closes the previous one) when
        ``self.record`` is set: per-region device time of one step without barriers or
        host syncs inside it (the reference's TimingReport regions, experiments/OGB/
        GCN.py:101-116, barriered and synced every region). CPU: host clock (the ops
        run synchronously)."""
        if not self.record:
            return
        if self.dev.type != "cuda":
            import time

            self._events.append((name, time.perf_counter()))
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self._events.append((name, ev))

    def region_ms(self) -> dict:
        """Milliseconds per region of the last recorded step (device time; host sync)."""
        if not self._events:
            return {}
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)
        out: dict = {}
        for (name, a), (_, b) in zip(self._events[:-1], self._events[1:]):
            dt = a.elapsed_time(b) if self.dev.type == "cuda" else (b - a) * 1e3
            out[name] = out.get(name, 0.0) + dt
        return out

    def check_errors(self) -> None:
        """Raise if a fused-kernel synchronisation wait timed out (host sync)."""
        if self.fwd_err is not None and int(self.fwd_err.item()) != 0:
            raise RuntimeError("FusedSAGE: sage_fwd_f32 role synchronisation timed out")

    @property
    def edges_aggregated(self) -> int:
        return self.g.edges_aggregated

    @edges_aggregated.setter
    def edges_aggregated(self, v: int) -> None:
        self.g.edges_aggregated = v

    # ------------------------------------------------------------------ helpers
    def _gemm(self, A1, B1, A2=None, B2=None, **kw):
        """fp32 dual GEMM: exact-f32 MFMAs, or bf16x3 split products with the weights split
        once per step (``GEMM_X3``)."""
        if self.x3:
            kw["b1x3"] = self._split(B1)
            if B2 is not None:
                kw["b2x3"] = self._split(B2)
        return F32.gemm_f32(A1, B1, A2, B2, **kw)

    def _split(self, B):
        # keyed by address; the entry keeps B alive, so no other tensor can take its address
        # while the cache (one step) lives
        key = (B.data_ptr(), tuple(B.shape), B.stride())
        v = self._x3_cache.get(key)
        if v is None:
            v = (B, F32.split_x3(B))
            self._x3_cache[key] = v
        return v[1]

    def _spmm(self, rowptr, col, x, out=None, **kw):
        """fp32 SpMM at the column-pass width tuned for ``x``'s width (``_tune_passes``)."""
        kw.setdefault("pass_cols", self.pass_for.get(x.shape[1], 0))
        return F32.spmm_f32(rowptr, col, x, out, **kw)

    def _tune_passes(self) -> None:
        """Column-pass width per operand width, from the graph's locality: on a graph whose
        neighbour lists stay near the row (most entries within +-2^16 ids), narrow
        (64-column) passes keep each pass's window of neighbour rows in the L2 / Infinity
        Cache (13.1 TB/s effective vs 9.8 at 128 columns on the bench graph); on a graph
        without that locality every neighbour row is a random HBM access and full-width
        passes read each row once, in one burst, instead of once per pass (structureless
        papers100M step 5508 -> 3687 ms, profiles/r03/). The locality is the fraction of
        the entries of 65536 evenly spaced rows within +-min(2^16, n/64) of their row (a timing-based
        choice on one chunk proved noisy). DGRAPH_FUSED_PASS_COLS forces a width."""
        self.pass_for = {}
        self.locality = None
        forced = int(os.environ.get("DGRAPH_FUSED_PASS_COLS", "0"))
        if forced:
            self.pass_for = {self.d0: min(forced, self.d0), self.hid: min(forced, self.hid)}
            return
        if self.dev.type != "cuda":
            return
        it = self.it
        n = self.L
        rows = torch.linspace(0, n - 1, steps=min(n, 65536), device=self.dev).long()
        beg = it.rowptr[rows]
        deg = (it.rowptr[rows + 1] - beg).clamp_max(64)
        tot = int(deg.sum())
        if tot == 0:
            return
        seg = torch.repeat_interleave(torch.arange(rows.numel(), device=self.dev), deg)
        off = torch.cumsum(deg, 0) - deg
        pos = beg[seg] + (torch.arange(tot, device=self.dev) - off[seg])
        dist_ = (it.col[pos].long() - rows[seg]).abs()
        win = max(1024, min(1 << 16, n // 64))  # small graphs: a window relative to n
        self.locality = float((dist_ < win).float().mean())
        for w in (self.d0, self.hid):
            self.pass_for[w] = 64 if self.locality >= 0.5 else w

    @staticmethod
    def _halo_range(csr, r0: int, r1: int):
        """Rows [k0, k1) of a row-compacted CSR whose output rows fall in [r0, r1), with
        their chunk-local output rows."""
        if csr is None:
            return None
        rm = csr.row_map
        k0 = int(torch.searchsorted(rm, torch.tensor(r0, device=rm.device)))
        k1 = int(torch.searchsorted(rm, torch.tensor(r1, device=rm.device)))
        if k1 <= k0:
            return None
        return (csr.rowptr[k0:k1 + 1], (rm[k0:k1] - r0).contiguous(), k1 - k0)

    def _agg_chunk(self, xin: torch.Tensor, xhalo: Optional[torch.Tensor], ci: int,
                   out: torch.Tensor, gate=None) -> torch.Tensor:
        """``out[:n] = mean over in-neighbours of rows chunk ci`` (interior + halo)."""
        r0, r1 = self.chunks[ci]
        n = r1 - r0
        o = out[:n]
        it = self.it
        self._spmm(it.rowptr[r0:r1 + 1], it.col, xin, o, row_scale=self.inv_deg[r0:r1],
                     gate=gate)
        hr = self.ch_halo[ci]
        if xhalo is not None and hr is not None:
            rp, rmap, _ = hr
            self._spmm(rp, self.hcomp.col, xhalo, o, row_scale=self.inv_deg[r0:r1], beta=1.0,
                         row_map=rmap, gate=gate)
        return o

    def _exchange(self, h: torch.Tensor):
        """Start the halo rows of ``h`` on their way from their owners (forward all-to-all-v,
        asynchronous): ``(recv, work)``, or None at W=1."""
        g = self.g
        if g.halo is None:
            return None
        return g.a2a(K.gather_rows(h, g.send_map.idx), async_op=True)

    def _layer(self, hin: torch.Tensor, halo, consume, width: int, name: str,
               store: Optional[torch.Tensor] = None):
        """Aggregate every row chunk of ``hin`` (interior + halo part) and hand it to
        ``consume(ci, agg, k)``. ``halo``: None (W=1), the received halo rows, or a pending
        ``(recv, work)`` exchange. With a pending exchange and the whole-layer aggregate
        buffer, the interior aggregation of all chunks runs first — while the halo rows are
        on the links — then the exchange is waited for and the halo parts and the GEMMs
        follow chunk by chunk. ``store`` (an [L, >= width] buffer that is free until the
        consumer writes row chunk c, e.g. the layer's own output: the GEMM of chunk c reads
        its aggregate rows before it overwrites them, tile by tile) stands in for the
        whole-layer buffer when there is no room for one. Returns the halo rows (for the
        backward)."""
        items = [ci for ci, (r0, r1) in enumerate(self.chunks) if r1 > r0]
        if store is None and self.agg_full is not None:
            store = self.agg_full
        if isinstance(halo, tuple) and store is not None:
            recv, work = halo
            af = store[:, :width]
            it = self.it
            for ci in items:
                r0, r1 = self.chunks[ci]
                self._spmm(it.rowptr[r0:r1 + 1], it.col, hin, af[r0:r1],
                             row_scale=self.inv_deg[r0:r1])
            self._mark(f"exchange_{name}")
            work.wait()
            self._mark(name)

            def produce(ci, k):
                r0, r1 = self.chunks[ci]
                hr = self.ch_halo[ci]
                if hr is not None:
                    rp, rmap, _ = hr
                    self._spmm(rp, self.hcomp.col, recv, af[r0:r1], beta=1.0, row_map=rmap,
                                 row_scale=self.inv_deg[r0:r1])
                return af[r0:r1]

            self.pipe.run(items, produce, consume)
            return recv
        if isinstance(halo, tuple):
            recv, work = halo
            self._mark(f"exchange_{name}")
            work.wait()
            self._mark(name)
            halo = recv

        def produce(ci, k):
            return self._agg_chunk(hin, halo, ci, self.bufA2[k][:, :width])

        self.pipe.run(items, produce, consume)
        return halo

    def _params(self):
        out = []
        for l in self.model.layers:
            out.append((l.w_self, l.w_neigh, l.bias))
        return out

    def _pad_in(self, w: torch.Tensor) -> torch.Tensor:
        """A layer-0 weight [d0_in, hid] as the [d0, hid] operand of the padded input."""
        w = w.detach()
        if self.d0 == self.d0_in:
            return w.contiguous()
        wp = torch.zeros(self.d0, w.shape[1], dtype=w.dtype, device=w.device)
        wp[:self.d0_in] = w
        return wp

    # ------------------------------------------------------------------ the step
    def step(self) -> torch.Tensor:
        g, x = self.g, self.x
        nl, hid, C, Cp, Cg = self.nl, self.hid, self.C, self.Cp, self.Cg
        P = self._params()
        dev = self.dev
        self._events = []
        self._x3_cache = {}  # weights changed since the last step: split again
        self._mark("fwd_l0")
        nnz_it = self.it.nnz
        nnz_h = self.halo.nnz if self.halo is not None else 0
        # ---------------- forward: hidden layers
        hin, hin_halo = x, (g._static_halo(x) if g.halo is not None else None)
        halos = []
        for l in range(nl - 1):
            ws, wn, b = P[l]
            if l == 0:
                ws, wn = self._pad_in(ws), self._pad_in(wn)
            else:
                ws, wn = ws.detach().contiguous(), wn.detach().contiguous()
            hout = self.h[l]
            bias = b.detach()

            def consume(ci, a, k, hin=hin, hout=hout, ws=ws, wn=wn, bias=bias):
                r0, r1 = self.chunks[ci]
                self._gemm(hin[r0:r1], ws, a, wn, bias=bias, relu=True, out=hout[r0:r1])

            if self.fwd_ring is not None and not self.x3 and hin.shape[1] in (128, 256):
                # aggregation + combine of the whole layer in one kernel
                it = self.it
                _native.ops().sage_fwd_f32(hin, it.rowptr, it.col, self.inv_deg, ws, wn,
                                           bias.float().contiguous(), hout, self.fwd_ring,
                                           self.fwd_err)
                halos.append(None)
            else:
                # layer l >= 1 can aggregate in place in its own output buffer (same width)
                inplace = hout if (OVERLAP_FWD and l > 0 and hin.shape[1] == hout.shape[1]) \
                    else None
                halos.append(self._layer(hin, hin_halo, consume, hin.shape[1], f"fwd_l{l}",
                                         store=inplace))
            self.edges_aggregated += nnz_it + nnz_h
            hin = hout
            # this layer's halo rows leave now and land while the next layer aggregates
            hin_halo = self._exchange(hout)
            self._mark(f"fwd_l{l + 1}" if l + 1 < nl - 1 else "fwd_out")
        # ---------------- forward: output layer (all rows), loss and eval on the fly
        ws, wn, b = P[nl - 1]
        wsp = torch.zeros(hid, Cp, device=dev)
        wsp[:, :C] = ws.detach()
        wnp = torch.zeros(hid, Cp, device=dev)
        wnp[:, :C] = wn.detach()
        bp = torch.zeros(Cp, device=dev)
        bp[:C] = b.detach()
        self.acc_out_s.reset()
        self.acc_out_n.reset()
        hl = hin
        hl_halo = self._layer(hl, hin_halo, lambda ci, a, k: self._out_chunk(ci, a, k, hl, wsp,
                                                                             wnp, bp),
                              hid, "fwd_out")
        halos.append(hl_halo)
        self.edges_aggregated += nnz_it + nnz_h
        # per-row losses / hits summed once, in a fixed order
        loss = self.row_loss.sum() * self.inv_n
        hv = self.hit.long()
        self.correct[0] = (hv * self.E_val_l).sum()
        self.correct[1] = (hv * (1 - self.E_val_l)).sum()
        self._mark("bwd_out")
        return self._backward(P, halos, hl, hl_halo, loss, nnz_it, nnz_h)

    def _out_chunk(self, ci, a, k, hl, wsp, wnp, bp):
        """Output layer of row chunk ci (consumer stream): logits of every row, the loss
        rows' cross-entropy gradient and output-layer weight gradients, eval hits."""
        C, Cp = self.C, self.Cp
        r0, r1 = self.chunks[ci]
        n = r1 - r0
        z = self._gemm(hl[r0:r1], wsp, a, wnp, bias=bp, out=self.bufB2[k][:n, :Cp])
        t0, t1 = self.ch_T[ci]
        if t1 > t0:
            # one fused kernel: per-row loss and the scaled softmax gradient rows
            tl = self.ch_Tloc[ci]
            dzt = self.dz[t0:t1]
            F32.xent_rows(z, tl, self.yT[t0:t1], self.inv_n, dzt, self.row_loss[t0:t1], C)
            self.acc_out_s.add(hl, dzt, a1_rows=self.T[t0:t1])
            self.acc_out_n.add(a, dzt, a1_rows=tl)
        e0, e1 = self.ch_E[ci]
        if e1 > e0:
            F32.argmax_hits(z, self.ch_Eloc[ci], self.yE[e0:e1], self.hit[e0:e1], C)

    def _backward(self, P, halos, hl, hl_halo, loss, nnz_it, nnz_h):
        g, x, dev = self.g, self.x, self.dev
        nl, hid, C, Cg = self.nl, self.hid, self.C, self.Cg
        ws, wn, _ = P[nl - 1]
        # ---------------- backward: output layer -> dZ of the last hidden layer on S
        hlast = hl
        F32.row_keep_bits(hlast, self.S, self.bits)  # the last hidden ReLU derivative on S
        del hl_halo, halos[-1]
        gw = {}
        dws2 = self.acc_out_s.result()[:, :C]
        dwn2 = self.acc_out_n.result()[:, :C]
        gw[(nl - 1, 0)], gw[(nl - 1, 1)] = dws2, dwn2
        gw[(nl - 1, 2)] = K.col_sum(self.dz)[:C]
        wn_t = torch.zeros(Cg, hid, device=dev)
        wn_t[:C] = wn.detach().t()
        ws_t = torch.zeros(Cg, hid, device=dev)
        ws_t[:C] = ws.detach().t()
        u2 = self._gemm(self.dz, wn_t, row_scale=self.invdegT, out=self.u_out)
        dZ = self.dZ
        work = None
        if self.sub is not None:
            ht_nz, a2a_sub, stc, stc_rows = self.sub
            hg = self._spmm(ht_nz.rowptr, ht_nz.col, u2)
            sg, work = a2a_sub(hg, async_op=True)
            self.edges_aggregated += ht_nz.nnz
        self._spmm(self.AT_S.rowptr, self.AT_S.col, u2, dZ)
        self.edges_aggregated += self.AT_S.nnz
        if work is not None:
            self._mark("exchange_bwd_out")
            work.wait()
            self._mark("bwd_out")
            self._spmm(stc.rowptr, stc.col, sg, dZ, beta=1.0, row_map=stc_rows)
            del sg, hg
        self._gemm(self.dz, ws_t, cin=dZ, o_rows=self.posT, out=dZ)
        F32.apply_keep_bits(dZ, self.bits)
        # ---------------- backward: last hidden layer (index nl-2) weights over S rows
        lh = nl - 2
        self._mark(f"bwd_l{lh}")
        ws1, wn1, _ = P[lh]
        hin_l = x if lh == 0 else self.h[lh - 1]
        hin_l_halo = halos[lh]
        gw[(lh, 2)] = K.col_sum(dZ)
        u = None
        work = None
        if nl == 3:
            # u1 = (dZ1 Wn1^T) / deg_S: its transposed aggregation feeds layer 0; the halo
            # part is computed and sent first so the exchange overlaps the S-row work below
            u = self._gemm(dZ, wn1.detach().t().contiguous(), row_scale=self.invdegS,
                             out=self.u)
            if self.haloT is not None:
                hg1 = self._spmm(self.haloT.rowptr, self.haloT.col, u, col_map=self.smap)
                sg1, work = g.a2a_rev(hg1, async_op=True)
                self.edges_aggregated += self.haloT.nnz
        self.acc_hid_s.reset()
        self.acc_hid_n.reset()
        def produce_s(sr, k):
            s0, s1 = sr
            rows = self.S[s0:s1]
            aS = self.bufA2[k][:s1 - s0, :hin_l.shape[1]]
            self._spmm(self.it.rowptr, self.it.col, hin_l, aS, row_ids=rows,
                         row_scale=self.invdegS[s0:s1])
            if hin_l_halo is not None:
                self._spmm(self.halo.rowptr, self.halo.col, hin_l_halo, aS, row_ids=rows,
                             row_scale=self.invdegS[s0:s1], beta=1.0)
            return aS

        def consume_s(sr, aS, k):
            s0, s1 = sr
            self.acc_hid_s.add(hin_l, dZ[s0:s1], a1_rows=self.S[s0:s1])
            self.acc_hid_n.add(aS, dZ[s0:s1])

        self.pipe.run([sr for sr in self.s_chunks if sr[1] > sr[0]], produce_s, consume_s)
        self.edges_aggregated += self.nnz_S
        gw[(lh, 0)] = self.acc_hid_s.result()
        gw[(lh, 1)] = self.acc_hid_n.result()
        if lh == 0:
            gw[(0, 0)], gw[(0, 1)] = gw[(0, 0)][:self.d0_in], gw[(0, 1)][:self.d0_in]
        if nl == 3:
            # ------------ layer 0: dZ0 by row chunks, consumed at once by its weight grads
            ws1_t = ws1.detach().t().contiguous()
            if work is not None:
                self._mark("exchange_bwd_l0")
                work.wait()
            self._mark("bwd_l0")
            self.acc_in.reset()
            db0s = []
            h1 = self.h[0]
            x_halo = halos[0]
            # the support rows' own term dZ1 Ws1^T, once over S (one full-size GEMM instead
            # of a row-scattered one per chunk); added by the aggregation's epilogue
            v = self._gemm(dZ, ws1_t, out=self.v_self) if self.v_self is not None else None

            def produce_0(ci, k):
                # memory-bound: the column-mapped transposed aggregation of u1 (gated by
                # layer 0's ReLU) and the recomputed layer-0 input aggregate
                r0, r1 = self.chunks[ci]
                n = r1 - r0
                gz = self.bufB2[k][:n, :hid]
                self._spmm(self.it.rowptr[r0:r1 + 1], self.it.col, u, gz, col_map=self.smap,
                             gate=h1[r0:r1], self_add=v,
                             self_map=self.smap if v is not None else None, self_row0=r0)
                sr = self.ch_send[ci]
                if work is not None and sr is not None:
                    rp, rmap, _ = sr
                    self._spmm(rp, self.send_st.col, sg1, gz, beta=1.0, row_map=rmap,
                                 gate=h1[r0:r1])
                a0 = self._agg_chunk(x, x_halo, ci, self.bufA2[k][:, :self.d0])
                return gz, a0

            def consume_0(ci, ga, k):
                gz, a0 = ga
                r0, r1 = self.chunks[ci]
                s0, s1 = self.ch_S[ci]
                if v is None and s1 > s0:  # no room for v_self: scattered self term
                    self._gemm(dZ[s0:s1], ws1_t, cin=gz, o_rows=self.ch_Sloc[ci],
                                 gate=h1[r0:r1], out=gz)
                self.acc_in.add(x[r0:r1], gz, A2=a0)
                db0s.append(K.col_sum(gz))

            self.pipe.run([ci for ci, (r0, r1) in enumerate(self.chunks) if r1 > r0],
                          produce_0, consume_0)
            db0 = torch.stack(db0s).sum(0) if db0s else torch.zeros(hid, device=dev)
            self.edges_aggregated += 2 * nnz_it + nnz_h + \
                (self.send_st.nnz if self.send_st is not None else 0)
            w0 = self.acc_in.result()
            gw[(0, 0)], gw[(0, 1)], gw[(0, 2)] = (w0[:self.d0_in],
                                                  w0[self.d0:self.d0 + self.d0_in], db0)
        self._mark("grads")
        # ---------------- gradients into the parameters
        for l, (ws_, wn_, b_) in enumerate(P):
            for k, p in enumerate((ws_, wn_, b_)):
                if p is None:
                    continue
                gk = gw[(l, k)].to(p.dtype).reshape(p.shape)
                if p.grad is None:
                    p.grad = gk.clone()
                else:
                    p.grad.copy_(gk)
        self._mark("end")
        return loss
