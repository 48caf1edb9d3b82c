"""Memory-lean fp32 full-graph GraphSAGE step (the headline config at the reference's
precision).

The reference trains in fp32 only (DGraph/distributed/csrc/torch_local_kernels.cu:43-46;
experiments/OGB/main.py:129-184 run the full-graph epoch: forward of every vertex, masked
loss, backward, optimizer step). At the ogbn-papers100M shape a plain fp32 layer-by-layer
autograd step needs ~420 GB on one GPU (features 57 GB, two hidden activations 114 GB each,
their aggregates and gradients as large). This executor is a hand-scheduled forward and
backward over ROW CHUNKS that never materialises an aggregate, a logit matrix or a dense
hidden gradient:

forward (per row chunk c, every vertex of every layer):
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
gates / two sources (csrc/kernels/spmm_f32.hip), MFMA f32 dual GEMM with
bias/ReLU/gate/row-scatter epilogues (gemm_f32.hip), split-M MFMA weight gradients
(wgrad_f32.hip), keep bits (bits.hip). Deterministic: fixed chunking, fixed reduction
orders, no atomics.

Vertex-partitioned graphs (W > 1). The rank's adjacency is ONE array per row: its interior
entries (columns < L) then its halo entries (columns L + h), with a per-row split pointer,
so an aggregation reads interior and halo of a row in one pass when the halo rows are
resident (the input features' halo, exchanged once; the backward's S rows), and either part
alone when they are not. With rows numbered interior-first (parallel/reorder.py: rows
[0, L_int) have no halo neighbour and are sent to nobody), each forward layer whose halo
exchange is in flight runs its interior rows to completion — aggregation, GEMM, loss, eval —
then the interior part of its boundary rows into a store when one is free (the layer's own
output buffer, or the whole-layer aggregate buffer), then waits and finishes the boundary
rows; the backward's reverse exchange (B1b) overlaps the S-row work and the interior rows'
input-layer gradient. Received halo rows are part of the memory plan, which raises
MemoryError before allocating when a configuration cannot fit.

Measured choices (profiles/r03/, PERFORMANCE.md): the SpMM column-pass width follows the
graph's locality (64 columns on a windowed graph, full rows on a structureless one); the
column-mapped transposed aggregation compacts each chunk's mapped entries before gathering;
the chunks run on one stream (a two-stream pipeline and a one-kernel fused layer were
correct but not faster: the fp32 GEMM's register footprint keeps the memory-bound and the
MFMA-bound work from co-residing; both were removed, PERFORMANCE.md keeps the numbers).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch

from ..comm.alltoallv import AllToAllV
from ..ops import f32 as F32
from ..ops import kernels as K
from ..parallel.dist_graph import DistGraph
from ..parallel.reorder import graph_locality
from ..utils.config import ExecutorConfig

# Executor knobs: utils/config.py ExecutorConfig, resolved per FusedSAGE (env
# DGRAPH_FUSED_<FIELD> or an explicit config=). What each one does, and the measurements
# behind its default:
# rows per chunk of the row-chunked passes (0 = auto from free memory)
#   -> ExecutorConfig.chunk_rows
# W > 1: overlap each forward halo exchange with work that does not need it
#   -> ExecutorConfig.overlap
# keep layer 0's input aggregate mean_N(x) from the forward for the backward when the
# memory plan has room for it ("auto"), never ("off"), or require it ("on")
#   -> ExecutorConfig.keep_agg0
# W > 1, a forward layer whose exchange is in flight: after its interior rows, aggregate the
# interior part of the boundary rows into a store before waiting ("on"), or wait and run the
# boundary rows in one two-source pass ("off"); "auto" stores only when the modelled
# exchange outlasts the interior rows' work (the store costs a second pass over the boundary
# rows and a read-modify-write of their aggregates: ~10 ms per layer at W = 8)
#   -> ExecutorConfig.boundary_store
# keep the last hidden layer's input aggregate on the support rows S from the forward (the
# forward computes it for every row anyway) instead of re-aggregating the S rows in the
# backward (and, with streamed halos, re-fetching the halo in column blocks): auto = when
# the memory plan has room for nS x width floats (always with streamed halos, whose plan
# already holds that store). Saves a pass over the S rows' entries per step.
#   -> ExecutorConfig.keep_as
# streamed hidden layers: the self term h W_self + b as a separate GEMM during the first
# column block's transfer (1), or the dual GEMM after the aggregation, in place (0)
#   -> ExecutorConfig.stream_fill
# streamed halos: the first column block half as wide as the rest (the pipeline fill, whose
# transfer nothing but the fill work hides, is half as long). Off: the extra column pass
# costs what it saves (W=8 structureless rank 700.6 ms with, 698.8 without; exposed
# exchange 15 vs 53 ms, profiles/r05/rehearse_structureless_ramp_zself.jsonl)
#   -> ExecutorConfig.stream_ramp
# streamed output layer: its self term as a separate GEMM during the first block's transfer
# (into an [L, Cp] store, when it fits). Off: the split GEMM's extra store traffic costs
# what it hides (W=8 structureless fwd_out + its exchange 196 ms with, 191.5 without)
#   -> ExecutorConfig.stream_out_fill
# W > 1: hidden-layer halos exchanged and consumed in column blocks ("stream") instead of
# kept at full width for the whole step — "auto" when the full-width plan does not fit (a
# structureless graph's halo is nearly every remote vertex), "on" / "off" to force
#   -> ExecutorConfig.halo_stream
# input-layer backward: the transposed aggregation of u (stored on the support rows S only)
# over an adjacency compacted to the S columns once, with the columns already mapped to S
# positions (a plain SpMM over ~S/L of the entries), instead of the column-mapped pass over
# every entry — when the memory plan has room for it (auto), always (on) or never (off,
# the default). Against the column-mapped pass at 64-column passes it cut the W=2/4/8 rank
# step by 3-5 %; against the column-mapped pass at full width (_spmm_u) it is a tie
# (W=8 265.6-267.6 vs 267.0 ms, W=2 1062-1068 vs 1065 ms) at a few GB more memory.
#   -> ExecutorConfig.compact_t
# W > 1: where the halo pack (the gather of the send rows into the send buffer) runs: on the
# compute stream just before the exchange is issued ("compute"), or on the communication
# stream next to the exchange ("comm"). A pack co-running with the aggregation saturates
# HBM with the SpMM's loads behind it (the first column pass after it: 13.2 instead of
# 1.2 ms) and hides nothing: windowed W=8 rank 256.2 (comm) vs 257.1 ms (compute), W=2
# 976.5 vs 975.7; structureless W=8 682.8 vs 670.6 ms, exposed exchange 59.6 vs 12.5 ms
# (the streamed blocks' transfers start a pack earlier; profiles/r05/pack_ab.jsonl)
#   -> ExecutorConfig.pack_stream
# W > 1, resident halos: the pack fused into the GEMM that produces the sent rows (its
# epilogue also stores each row at its send-buffer positions) instead of a gather pass
#   -> ExecutorConfig.pack_fused
# W > 1, symmetric graph, 3 layers: the halo part of the input layer's backward aggregation
# A^T u (u = the layer-1 pre-activation gradient, nonzero on the support rows S only) by
# "pull" — the owners send their S rows of u that are some rank's halo rows (a forward-style
# exchange restricted to S), each rank aggregates them with its own rows in one two-source
# pass — or by "push": every rank aggregates the contributions of its rows to EVERY halo row
# (a transposed pass over H rows) and sends them back to the owners, who add them
#   -> ExecutorConfig.bwd_halo
# W > 1: the output layer projected BEFORE it is aggregated, when its padded width Cp is
# narrower than the hidden width (mean_N(h) W_neigh = mean_N(h W_neigh)): the logits'
# neighbour term aggregates and exchanges Cp columns instead of hid (172 -> 176 vs 256 on
# papers100M). "auto": when the plan has room for the [L, Cp] projection (the W_neigh
# weight gradient then needs the loss rows' aggregate of h, pulled separately: small)
#   -> ExecutorConfig.project_first
# column-mapped gradient SpMMs run full-width passes while the support S is at most this
# share of the rows (papers100M 0.28 at W=1 and W=8: full width, step 1865 ms / 266 ms;
# ogbn-products 0.98: 64-column passes, 71.7 vs 76.1 ms at full width)
#   -> ExecutorConfig.u_full_frac
# (column block, ring buffers) in order of preference: two buffers before wider blocks —
# with one buffer every block's transfer is exposed (a W=2 structureless rank: 1.1 s of its
# 3.1 s step), and 32-column passes aggregate at the 64-column rate per byte
# (profiles/r05/xcd_ab2.log)
#   -> ExecutorConfig.stream_shapes
# planning rates of the "auto" choice: xGMI per link and direction, fp32 SpMM gather
# (effective) and fp32 MFMA GEMM rates measured on MI355X (PERFORMANCE.md)
#   -> ExecutorConfig.plan_link_gbps
PLAN_LINK_GBPS = 153.0  # xGMI per link and direction: the planner's fallback rate
PLAN_SPMM_TBPS = 13.0   # row-group SpMM, 64-column passes, bench graph (PERFORMANCE.md)
PLAN_GEMM_TFPS = 120.0  # exact-f32 MFMA GEMM, interleaved with aggregations
PLAN_HBM_TBPS = 5.0     # streaming read-modify-write of a store


def _ranges(a: int, b: int, step: int) -> List[Tuple[int, int]]:
    return [(r, min(b, r + step)) for r in range(a, b, step)]


def _pad_to(n: int, m: int) -> int:
    return (n + m - 1) // m * m


HIDDEN_WIDTHS = (128, 256, 384, 512)  # multiples of 128: wgrad K-blocks, GEMM N-blocks
MAX_IN_WIDTH = 1024


def supported(model, x: torch.Tensor) -> bool:
    """Shapes the fused executor runs: 2 or 3 mean-aggregating layers, no dropout, hidden
    width in HIDDEN_WIDTHS (wider products run as several kernel tiles), input width up to
    MAX_IN_WIDTH (zero-padded to the kernels' multiple), at most 256 classes."""
    layers = list(model.layers)
    if len(layers) not in (2, 3) or getattr(model, "dropout", 0.0) != 0.0:
        return False
    hid = layers[0].out_dim
    d0 = x.shape[1]
    return (x.dtype == torch.float32 and 0 < d0 <= MAX_IN_WIDTH
            and hid in HIDDEN_WIDTHS and all(l.out_dim == hid for l in layers[:-1])
            and 0 < layers[-1].out_dim <= 256)


def _in_width(d0: int, nl: int = 3) -> int:
    """Input width the kernels run at (zero-padded features): the layer-0 GEMM's K (a
    multiple of 32), the input weight gradient's K = 2 * width (3 layers: a multiple of
    128) or K = width (2 layers: a multiple of 128)."""
    if nl == 3:
        return 64 if d0 <= 64 else _pad_to(d0, 64)
    return _pad_to(d0, 128)


def _width_at_least(c: int, widths) -> int:
    for w in widths:
        if w >= c:
            return w
    raise ValueError(f"no kernel width >= {c}")


def _compact_by_map(rowptr: torch.Tensor, col: torch.Tensor, rowend: Optional[torch.Tensor],
                    cmap: torch.Tensor, nrows: int, count_only: bool = False):
    """Entries ``[rowptr[r], rowend[r] or rowptr[r + 1])`` of rows ``r < nrows`` whose column
    maps (``cmap[c] >= 0``), in entry order, with the column replaced by ``cmap[c]``:
    ``(rowptr int64 [nrows + 1], col int32)``. Row chunks of ~2^26 entries (bounded
    temporaries). ``count_only``: just the number of kept entries."""
    dev = col.device
    start = rowptr[:nrows]
    deg = (rowend[:nrows] if rowend is not None else rowptr[1:nrows + 1]) - start
    total = int(deg.sum())
    step = max(1, int(nrows * (1 << 26) // max(total, 1)))
    chunks = [(r0, min(nrows, r0 + step)) for r0 in range(0, nrows, step)]

    def entries(r0, r1):
        d = deg[r0:r1]
        n = int(d.sum())
        if n == 0:
            return None, None
        rows = torch.repeat_interleave(torch.arange(r1 - r0, device=dev), d, output_size=n)
        first = torch.cumsum(d, 0) - d
        pos = start[r0:r1][rows] + torch.arange(n, device=dev) - first[rows]
        m = cmap[col[pos].long()]
        return rows, m

    counts = torch.zeros(nrows, dtype=torch.long, device=dev)
    for r0, r1 in chunks:
        rows, m = entries(r0, r1)
        if rows is not None:
            counts[r0:r1] = torch.bincount(rows[m >= 0], minlength=r1 - r0)
    if count_only:
        return int(counts.sum())
    rp = torch.zeros(nrows + 1, dtype=torch.long, device=dev)
    torch.cumsum(counts, 0, out=rp[1:])
    del counts
    out = torch.empty(int(rp[-1]), dtype=torch.int32, device=dev)
    for r0, r1 in chunks:
        rows, m = entries(r0, r1)
        if rows is not None:
            out[int(rp[r0]):int(rp[r1])] = m[m >= 0].to(torch.int32)
    return rp, out


class _Adj:
    """A rank's adjacency in one column array: row r's interior entries (columns < L) are
    ``col[rp[r]:mid[r]]``, its halo entries (columns L + h, h a received halo row) are
    ``col[mid[r]:rp[r + 1]]``. Without a halo ``mid`` is None and the array is the interior
    CSR itself (no copy)."""

    def __init__(self, interior, halo, L: int):
        self.L = L
        if halo is None or halo.nnz == 0 and halo.num_rows == 0:
            self.rp, self.col, self.mid = interior.rowptr, interior.col, None
            self.nnz_int, self.nnz_halo = interior.nnz, 0
            return
        dev = interior.device
        ideg = interior.rowptr[1:] - interior.rowptr[:-1]
        hdeg = halo.rowptr[1:] - halo.rowptr[:-1]
        rp = interior.rowptr + halo.rowptr
        mid = (rp[:-1] + ideg).contiguous()
        nnz = int(rp[-1])
        if L + int(halo.num_cols) >= 2 ** 31:
            raise ValueError("_Adj: local + halo rows must fit int32 column ids")
        col = torch.empty(nnz, dtype=torch.int32, device=dev)
        # chunked scatter of both parts (bounded temporaries at 10^9+ entries)
        step = max(1, int(L * (1 << 26) // max(nnz, 1)))
        for r0 in range(0, L, step):
            r1 = min(L, r0 + step)
            for src, deg, base, off in ((interior, ideg, rp, 0), (halo, hdeg, mid, L)):
                a, b = int(src.rowptr[r0]), int(src.rowptr[r1])
                if b == a:
                    continue
                shift = torch.repeat_interleave(base[r0:r1] - src.rowptr[r0:r1], deg[r0:r1],
                                                output_size=b - a)
                dst = torch.arange(a, b, device=dev, dtype=torch.long).add_(shift)
                del shift
                col[dst] = (src.col[a:b].to(torch.int32) + off) if off else \
                    src.col[a:b].to(torch.int32)
                del dst
        self.rp, self.col, self.mid = rp.contiguous(), col, mid
        self.nnz_int, self.nnz_halo = interior.nnz, halo.nnz

    @property
    def nnz(self) -> int:
        return self.nnz_int + self.nnz_halo

    def halo_degree(self) -> torch.Tensor:
        if self.mid is None:
            return torch.zeros(self.rp.numel() - 1, dtype=torch.long, device=self.rp.device)
        return self.rp[1:] - self.mid

    def rows(self, r0: int, r1: int, part: str):
        """(rowptr, rowend) kernel arguments of rows [r0, r1): ``part`` "all" (interior and
        halo entries), "int" (interior only) or "halo" (halo only)."""
        if self.mid is None or part == "all":
            if part == "halo":
                raise ValueError("no halo entries")
            return self.rp[r0:r1 + 1], None
        if part == "int":
            return self.rp[r0:r1], self.mid[r0:r1]
        return self.mid[r0:r1], self.rp[r0 + 1:r1 + 1]

    def memory_bytes(self) -> int:
        if self.mid is None:
            return 0  # the interior CSR's own arrays
        return self.rp.numel() * 8 + self.mid.numel() * 8 + self.col.numel() * 4


class _Budget:
    """The setup's device-memory plan (``FusedSAGE._plan_memory``): ``free`` bytes,
    ``need_h`` (activations and halo rows), ``other`` (workspaces and every buffer chosen so
    far), the ``margin`` an optional buffer must leave, the chunk arena's row widths
    (``wA`` aggregate, ``wB`` logit / gradient) and the sub-plan exchange's bytes."""

    def __init__(self, free: int, need_h: int, other: int, margin: int, wA: int, wB: int):
        self.free, self.need_h, self.other, self.margin = free, need_h, other, margin
        self.wA, self.wB = wA, wB
        self.sub_bytes = 0
        self.decisions: list = []

    def note(self, what: str, nbytes: int, taken: bool) -> None:
        """Record one plan choice with the room it was decided against (schedule())."""
        self.decisions.append({"what": what, "gb": round(nbytes / 2**30, 2),
                               "room_gb": round(self.room() / 2**30, 2), "taken": bool(taken)})

    def room(self) -> int:
        """Bytes not yet planned."""
        return self.free - self.need_h - self.other

    def describe(self, halo_bytes: int, dev) -> str:
        return (f"FusedSAGE: activations {self.need_h / 2**30:.1f} GiB (halo rows "
                f"{halo_bytes / 2**30:.1f}) + workspace {self.other / 2**30:.1f} GiB exceed the "
                f"{self.free / 2**30:.1f} GiB free on {dev}")


class FusedSAGE:
    """The fp32 training step of a 2- or 3-layer :class:`~dgraph_amd.models.sage.GraphSAGE`
    (mean aggregator, ReLU between layers, no dropout) over a :class:`DistGraph`.

    ``step()`` runs forward + backward, leaves the weight gradients in ``p.grad`` of the
    model's parameters and returns the loss (device scalar, this rank's share of the global
    mean: the sum over this rank's loss rows divided by the GLOBAL train-row count
    ``n_train``, so an all-reduce of the gradients gives the full-batch gradient).
    ``self.correct`` holds (validation hits, test hits) of the same forward.

    ``release_graph=True``: the graph's interior / halo CSRs are dropped once this
    executor has built its own adjacency (DistGraph.release_csr) — the graph object is then
    only an exchange plan."""

    def __init__(self, model, graph: DistGraph, x: torch.Tensor, train_idx: torch.Tensor,
                 y_train: torch.Tensor, eval_idx: torch.Tensor, y_eval: torch.Tensor,
                 eval_is_val: torch.Tensor, n_train: int, chunk_rows: int = 0,
                 release_graph: bool = False, reserve_bytes: int = 0,
                 config: Optional[ExecutorConfig] = None):
        if not supported(model, x):
            raise ValueError("FusedSAGE: unsupported model/feature shape")
        # the schedule knobs, resolved now (environment read at construction, not import)
        self.cfg = config if config is not None else ExecutorConfig.from_env()
        dev = x.device
        self.dev = dev
        if dev.type == "cuda":
            from .. import _native

            with torch.cuda.device(dev):
                # the persistent kernels' work-counter slots, before any graph capture
                _native.ops().f32_init()
            if os.environ.get("DGRAPH_F32_DYNAMIC") is not None:
                _native.ops().set_f32_sched(-1, int(os.environ["DGRAPH_F32_DYNAMIC"]))
        self.d0_in = x.shape[1]
        self.d0 = _in_width(self.d0_in, len(model.layers))
        if self.d0 != self.d0_in:
            # zero feature columns: their aggregates are zero, their weight rows get
            # gradients that are dropped (ogbn-products: 100 -> 128)
            xp = torch.zeros(x.shape[0], self.d0, dtype=x.dtype, device=dev)
            xp[:, :self.d0_in] = x
            x = xp
        self.model, self.g, self.x = model, graph, x.contiguous()
        self.L, self.H = graph.L, graph.H
        self.nl = len(model.layers)
        self.hid = model.layers[0].out_dim
        self.C = model.layers[-1].out_dim
        # logit GEMM width (N of the output GEMM) and the dz width (N of the output-layer
        # weight gradients, K of the projections of dz)
        self.Cp = _width_at_least(self.C, (64, 128, 176, 192, 256))
        self.Cg = _width_at_least(_pad_to(self.C, 32) if self.C > 128 else self.C,
                                  (128, 176, 192, 256))
        self.inv_n = 1.0 / max(int(n_train), 1)
        # setup phases: rows, adjacency (collective parts included), the memory plan (every
        # schedule choice, agreed over the plan's group), the row chunks, the buffers
        self._setup_rows(graph, train_idx, y_train, eval_idx, y_eval, eval_is_val)
        self._setup_adjacency(graph, release_graph)
        b = self._plan_memory(graph, reserve_bytes)
        self._plan_chunks(chunk_rows, b)
        self._allocate(graph, b)
        self.row_loss = torch.zeros(self.T.numel(), dtype=torch.float32, device=dev)
        self.hit = torch.zeros(self.E.numel(), dtype=torch.uint8, device=dev)
        self.E_val_l = self.E_val.long()
        self.correct = torch.zeros(2, dtype=torch.long, device=dev)
        self.record = False
        self._events: list = []
        self._packs: dict = {}  # send-row packs in source order (_pack)
        self._tune_passes()

    # ------------------------------------------------------------------ setup phases
    def _setup_rows(self, graph: DistGraph, train_idx, y_train, eval_idx, y_eval,
                    eval_is_val) -> None:
        """Loss / eval rows (sorted: chunk ranges are searchsorted) and the gradient support
        S (rows where dZ of the last hidden layer can be nonzero), with the output-layer
        backward's sub-plan when remote loss rows reach this rank."""
        dev, L = self.dev, self.L
        t, tp = torch.sort(train_idx.long())
        self.T, self.yT = t.contiguous(), y_train[tp].contiguous()
        e, ep = torch.sort(eval_idx.long())
        self.E, self.yE = e.contiguous(), y_eval[ep].contiguous()
        self.E_val = eval_is_val[ep].contiguous()
        self.inv_deg = graph.inv_deg
        self.invdegT = self.inv_deg[self.T].contiguous()
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
        if self.T.numel() and int(self.posT.min()) < 0:  # (T is part of S by construction)
            raise RuntimeError("FusedSAGE: a loss row outside the gradient support")
        self.invdegS = self.inv_deg[S].contiguous()
        self.AT_S = it_t.select_rows(S)            # rows S (compact), cols T (compact)
        del it_t
        self.sub = None
        self._sub_pull = None
        if sub is not None:
            ht_nz, a2a_sub, st = sub[0], sub[1], sub[2]
            stc = st.compact_rows()
            self.sub = (ht_nz, a2a_sub, stc, smap[stc.row_map].long().contiguous())
            # (my halo rows adjacent to a loss row, the rows of mine the peers' loss rows
            # neighbour: the project-first output layer pulls h over the reversed sub-plan)
            self._sub_pull = (sub[3], sub[4], a2a_sub)

    def _setup_adjacency(self, graph: DistGraph, release_graph: bool) -> None:
        """The one-array adjacency (interior + halo entries of a row), its transposed
        blocks, the pulled backward halo's plan and the link calibration (both collective,
        built by every rank before the memory plan can raise), and the interior prefix."""
        cfg, dev, L = self.cfg, self.dev, self.L
        it = graph.interior
        self.adj = _Adj(it, graph.halo, L)
        # B1b's transposed interior aggregation: the interior part of the rows themselves
        # when the interior block is symmetric, else its transpose
        self.itT = None if it.symmetric else it.transpose()
        self.pull = self._pull_plan(graph) \
            if (cfg.bwd_halo == "pull" and self.nl == 3 and graph.symmetric and
                graph.send_map is not None) else None
        # the per-peer link rate the overlap planner assumes: measured on this job's own
        # exchange (collective), not the xGMI peak
        self.link_gbps = self._calibrate_link(graph) if graph.send_map is not None \
            else PLAN_LINK_GBPS
        # the push path's transposed halo block and send-row scatter (not built for the
        # pull: at W=2 on the structureless graph the transposed halo alone is ~7 GB)
        push = self.pull is None and graph.halo is not None
        self.haloT = graph.halo.transpose() if push else None
        self.send_st = graph.send_map.transpose_csr().compact_rows() if push else None
        self.nnz_it, self.nnz_h = self.adj.nnz_int, self.adj.nnz_halo
        # entries of the S-row aggregation (B1a), counted on the host once
        self.nnz_S = int((self.adj.rp[self.S + 1] - self.adj.rp[self.S]).sum())
        # ---- interior prefix: rows [0, Li) have no halo entry and are sent to nobody
        bnd = self.adj.halo_degree() > 0
        if graph.send_map is not None and graph.send_map.idx.numel():
            bnd[graph.send_map.idx.long()] = True
        nzb = torch.nonzero(bnd)
        self.Li = int(nzb[0, 0]) if nzb.numel() else L
        del bnd, nzb
        self.locality = getattr(graph, "locality_hint", None)
        if self.locality is None and dev.type == "cuda":
            self.locality = graph_locality(self.adj.rp, self.adj.col, L)
        if release_graph:
            graph.release_csr()
            del it

    def _plan_memory(self, graph: DistGraph, reserve_bytes: int) -> "_Budget":
        """Every schedule choice, from the device's free memory: streamed halos and their
        shape, the kept aggregates, the projected output layer, the boundary stores, the
        pipeline-fill self term. Choices that change the sequence of collectives are agreed
        over the plan's group; a plan that does not fit raises MemoryError on every rank
        alike, before any allocation."""
        cfg, dev, L, H = self.cfg, self.dev, self.L, self.H
        # (the planning above left cached temporaries: return them first, and count what
        # the caching allocator still holds unused as free)
        if dev.type == "cuda":
            torch.cuda.empty_cache()
            free = torch.cuda.mem_get_info(dev)[0] + \
                torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
        else:
            free = 64 << 30
        # headroom the caller keeps out of the plan (a secondary measurement that must not
        # run the device to its last GB: rank-to-rank halo sizes and allocator rounding vary)
        free -= int(reserve_bytes)
        need_h = (self.nl - 1) * L * self.hid * 4
        self.store_sep = 2 * self.nS > L   # dZ and u do not fit in the last hidden buffer
        if self.store_sep:
            need_h += 2 * self.nS * self.hid * 4
        nT = self.T.numel()
        # dz rows, wgrad slabs, (u_out when it cannot live in the last hidden buffer) and
        # allocator / temporary slack; the chunk arena gets the rest
        self.u_sep = 2 * self.nS + nT > L
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count \
            if dev.type == "cuda" else 1
        kh = self.hid if self.nl == 3 else self.d0
        slab_floats = (2 * self.hid * self.Cg + 2 * kh * self.hid +
                       (2 * self.d0 * self.hid if self.nl == 3 else 0))
        other = 4 * nT * self.Cg + 4 * slab_floats * ncu * F32.WgradAcc.UNITS_PER_CU + \
            (3 << 29) + \
            (4 * nT * self.hid if self.u_sep else 0)
        b = _Budget(free, need_h, other, 16 << 30 if dev.type == "cuda" else 0,
                    wA=max(self.hid, self.d0), wB=max(self.Cp, self.hid))
        # W > 1: the received halo rows live through the step — the input's (exchanged once,
        # kept), every hidden layer's (the backward reads them) — and each exchange's send
        # rows while it is in flight: planned here, not discovered by the allocator
        n_send = graph.send_map.idx.numel() if graph.send_map is not None else 0
        self.n_send = n_send
        # the input's halo exchange (once, at the first step): its send/receive blocks live
        # next to everything planned here
        x_tr = 4 * (n_send + H) * graph.static_halo_block(self.d0) \
            if graph.send_map is not None else 0
        self.halo_bytes = 4 * (H * self.d0 + (self.nl - 1) * H * self.hid + n_send * self.hid)
        self.stream, self.cw, self.nbuf = False, 0, 0
        b.other += x_tr
        w_lh = self.d0 if self.nl == 2 else self.hid  # width of the last hidden layer's input
        self.w_lh = w_lh
        # the output-layer backward's sub-plan exchange (halo rows adjacent to the loss rows,
        # A[T, halo]^T u2 out, owners' rows back): resident buffers in storage that is dead
        # during that exchange — the last received-halo / send buffers, or the streamed ring
        self.sub_rows = (0, 0)
        if self.sub is not None:
            self.sub_rows = (self.sub[0].rowptr.numel() - 1, self.sub[1].total_recv)
        b.sub_bytes = 4 * self.hid * (self.sub_rows[0] + self.sub_rows[1])
        full_ok = dev.type != "cuda" or \
            b.need_h + self.halo_bytes + b.other + (1 << 28) <= b.free
        # Choices that change the SEQUENCE of collectives (streamed halos and their shape,
        # the projected output layer) are agreed over the plan's group: each rank plans from
        # its own free memory and partition sizes, and one rank choosing differently would
        # post all-to-all-v calls its peers never match (a hang or corrupted halos)
        want_stream = graph.send_map is not None and (
            cfg.halo_stream == "on" or (cfg.halo_stream == "auto" and not full_ok))
        if graph.send_map is not None:
            want_stream = bool(self._agree([int(want_stream)], "max")[0])
        if want_stream:
            # streamed halos: the input's halo stays resident (static), the hidden layers'
            # cross in column blocks of cw through a ring of nbuf send/receive buffers, and
            # whole-row aggregates land in stores (the output layer's, the S rows' of the
            # re-fetched h1, the reverse exchange's input-layer gradient)
            # (the reverse exchange's input-layer gradient store lives in the output
            # layer's aggregate store, dead once the forward is done)
            stores = L * max(self.hid, self.d0) * 4 + self.nS * w_lh * 4
            shapes = cfg.shapes()
            fit, hbs = [], []
            for cw, nb in shapes:
                ring = max(nb * (H + n_send) * cw * 4, b.sub_bytes)
                hb = 4 * H * self.d0 + ring + stores
                hbs.append(hb)
                fit.append(int(self.hid % cw == 0 and (
                    dev.type != "cuda" or b.need_h + hb + b.other + (1 << 28) <= b.free)))
            fit = self._agree(fit, "min")  # the first shape EVERY rank has room for
            for (cw, nb), ok, hb in zip(shapes, fit, hbs):
                b.note(f"halo_stream_{cw}x{nb}", hb, ok and not self.stream)
                if ok and not self.stream:
                    self.stream, self.cw, self.nbuf, self.halo_bytes = True, cw, nb, hb
        b.need_h += self.halo_bytes
        fits = dev.type != "cuda" or b.need_h + b.other + (1 << 28) <= b.free
        if graph.send_map is not None and not bool(self._agree([int(fits)], "min")[0]):
            # fail here, before any allocation (and after every collective of the setup), on
            # every rank alike, so a caller can skip the configuration instead of dying
            # mid-step
            raise MemoryError(b.describe(self.halo_bytes, dev) +
                              ("" if not fits else " of another rank of the group"))
        if not fits:
            raise MemoryError(b.describe(self.halo_bytes, dev))
        self._plan_compact_t(b)
        self._plan_compact_pull(b)
        # the last hidden layer's input aggregate on the S rows kept from the forward (else
        # re-aggregated in the backward); streamed halos keep it in aS_full (planned above)
        self.aS_keep = None
        need_as = self.nS * self.w_lh * 4
        self.keep_as = cfg.keep_as == "on" or self.stream or (
            cfg.keep_as == "auto" and b.room() - need_as > b.margin)
        b.note("keep_aS", 0 if self.stream else need_as, self.keep_as)
        if self.keep_as and not self.stream:
            b.other += need_as
        # layer 0's input aggregate kept from the forward for the backward (else recomputed)
        self.agg0 = None
        need0 = L * self.d0 * 4
        if self.nl == 3 and cfg.keep_agg0 != "off":
            take = cfg.keep_agg0 == "on" or b.room() - need0 > b.margin
            b.note("keep_agg0", need0, take)
            if take:
                self.agg0 = torch.empty(L, self.d0, dtype=torch.float32, device=dev)
                b.other += need0
        # W > 1: the output layer's projection [L, Cp] (PROJECT_FIRST), after the kept
        # aggregates (those save whole aggregation passes)
        self.pf = None
        need_pf = L * self.Cp * 4
        if graph.send_map is not None and cfg.project_first != "off" and self.Cp < self.hid:
            want_pf = cfg.project_first == "on" or b.room() - need_pf > b.margin
            want_pf = bool(self._agree([int(want_pf)], "min")[0])  # (changes the exchanges)
            b.note("project_first", need_pf, want_pf)
            if want_pf:
                self.pf = torch.empty(L, self.Cp, dtype=torch.float32, device=dev)
                b.other += need_pf
                self._aggT_setup()
        # W > 1: a whole-layer aggregate buffer lets the interior part of the OUTPUT layer's
        # boundary rows run while its halo rows are in flight (hidden layers use their own
        # output buffer for that). Planned after the kept aggregates: those save whole
        # aggregation passes, the store only exposed exchange time
        self.use_store = self._plan_store()
        self.agg_full = None
        need_full = (L - self.Li) * b.wA * 4
        if graph.send_map is not None and cfg.overlap and self.Li < L and not self.stream \
                and self.use_store["out"]:
            take = b.room() - need_full > b.margin
            b.note("output_store", need_full, take)
            if take:
                self.agg_full = torch.empty(L - self.Li, b.wA, dtype=torch.float32, device=dev)
                b.other += need_full
        # streamed output layer: its self term h W_self + b for every row, computed during
        # the first column block's transfer (the pipeline fill), when the plan has room
        self.zself = None
        need_z = L * self.Cp * 4
        if self.stream and cfg.stream_out_fill and self.pf is None:
            take = b.room() - need_z > b.margin
            b.note("output_self_term_fill", need_z, take)
            if take:
                self.zself = torch.empty(L, self.Cp, dtype=torch.float32, device=dev)
                b.other += need_z
        return b

    def _plan_compact_t(self, b: "_Budget") -> None:
        """The input-layer backward's S-compacted transposed adjacencies (COMPACT_T): built
        when they leave at least 1 GB for the chunk arena (they shrink the arena, not the
        plan)."""
        cfg, dev, L = self.cfg, self.dev, self.L
        self.TS = None
        if self.nl == 3 and cfg.compact_t != "off":
            if self.itT is not None:
                src = (self.itT.rowptr, self.itT.col, None)
            else:
                src = (self.adj.rp, self.adj.col, self.adj.mid)
            nnz_ts = _compact_by_map(src[0], src[1], src[2], self.smap, L, count_only=True) \
                if L else 0
            ts_bytes = nnz_ts * 4 + (L + 1) * 8
            take = cfg.compact_t == "on" or dev.type != "cuda" or \
                b.room() - (1 << 28) - ts_bytes >= (1 << 30)
            b.note("compact_T", ts_bytes, take)
            if take:
                self.TS = _compact_by_map(src[0], src[1], src[2], self.smap, L)
                b.other += ts_bytes
        # the same for the halo rows' transposed aggregation of u (the reverse exchange's
        # payload, computed before the S-row work so the exchange overlaps it)
        self.HTS = None
        if self.TS is not None and self.haloT is not None:
            Hn = self.haloT.rowptr.numel() - 1
            nnz_h = _compact_by_map(self.haloT.rowptr, self.haloT.col, None, self.smap, Hn,
                                    count_only=True)
            hts_bytes = nnz_h * 4 + (Hn + 1) * 8
            take = cfg.compact_t == "on" or dev.type != "cuda" or \
                b.room() - (1 << 28) - hts_bytes >= (1 << 30)
            b.note("compact_halo_T", hts_bytes, take)
            if take:
                self.HTS = _compact_by_map(self.haloT.rowptr, self.haloT.col, None, self.smap,
                                           Hn)
                b.other += hts_bytes

    def _plan_compact_pull(self, b: "_Budget") -> None:
        """The pulled backward halo's adjacency with its column map applied once (``PT``):
        only the entries whose neighbour is a support row (mine, or a peer's pulled in), with
        the mapped column (support index, or ``nS`` + pulled row) stored in place of the
        original. Streamed halos pull u in column blocks, and without it every block's pass
        of B1b walks ALL entries and looks each column up in the map (a random 4-byte read
        per entry per block): the structureless W=2 rank spent 58 ms per 32-column block
        there, for ~26 % of the entries used. A resident pull walks the map once, in one
        full-width pass (``_spmm_u``), so "auto" builds it for streamed halos only."""
        cfg, dev, L = self.cfg, self.dev, self.L
        self.PT = None
        if self.pull is None or cfg.compact_pull == "off" or not L or (
                cfg.compact_pull == "auto" and not self.stream):
            return
        nnz = _compact_by_map(self.adj.rp, self.adj.col, None, self.pull["cmap"], L,
                              count_only=True)
        nbytes = nnz * 4 + (L + 1) * 8
        take = cfg.compact_pull == "on" or dev.type != "cuda" or \
            b.room() - (1 << 28) - nbytes >= (1 << 30)
        b.note("compact_pull", nbytes, take)
        if take:
            self.PT = _compact_by_map(self.adj.rp, self.adj.col, None, self.pull["cmap"], L)
            b.other += nbytes

    def _plan_chunks(self, chunk_rows: int, b: "_Budget") -> None:
        """Row chunks sized from what the plan left (never straddling the interior /
        boundary split), with each chunk's loss / eval / support row ranges."""
        L = self.L
        spare = max(b.room(), 1 << 28)
        per_row = 4 * (b.wA + b.wB)  # aggregate + logit/gradient chunk buffers
        cr = chunk_rows or self.cfg.chunk_rows
        if cr <= 0:
            cr = int(min(max(spare // per_row, 1 << 16), 1 << 21))
        self.cr = max(256, min(int(cr), max(L, 256)))
        b.note("chunk_arena", self.cr * per_row, True)
        self.memory_plan = b.decisions
        self.chunks = _ranges(0, self.Li, self.cr) + _ranges(self.Li, L, self.cr)
        if not self.chunks:
            self.chunks = [(0, 0)]
        self.nA = sum(1 for r0, r1 in self.chunks if r1 <= self.Li and r1 > r0)
        self.s_chunks = _ranges(0, self.nS, self.cr) or [(0, 0)]
        ss = lambda v, a: int(torch.searchsorted(v, torch.tensor(a, device=v.device)))  # noqa
        self.ch_T = [(ss(self.T, r0), ss(self.T, r1)) for r0, r1 in self.chunks]
        self.ch_E = [(ss(self.E, r0), ss(self.E, r1)) for r0, r1 in self.chunks]
        self.ch_S = [(ss(self.S, r0), ss(self.S, r1)) for r0, r1 in self.chunks]
        self.ch_Tloc = [(self.T[a:b_] - r0).contiguous()
                        for (r0, _), (a, b_) in zip(self.chunks, self.ch_T)]
        self.ch_Eloc = [(self.E[a:b_] - r0).contiguous()
                        for (r0, _), (a, b_) in zip(self.chunks, self.ch_E)]
        self.ch_Sloc = [(self.S[a:b_] - r0).contiguous()
                        for (r0, _), (a, b_) in zip(self.chunks, self.ch_S)]
        self.ch_send = [self._csr_range(self.send_st, r0, r1) for r0, r1 in self.chunks]

    def _allocate(self, graph: DistGraph, b: "_Budget") -> None:
        """The persistent buffers the plan counted (allocated once: no allocation in the
        steady state)."""
        cfg, dev, L, H = self.cfg, self.dev, self.L, self.H
        n_send, nT = self.n_send, self.T.numel()
        f = dict(dtype=torch.float32, device=dev)
        self.h = [torch.empty(L, self.hid, **f) for _ in range(self.nl - 1)]
        # W > 1: the exchange buffers, resident — an exchange's buffers are in use on the
        # comm stream until it completes, so per-step buffers would make the caching
        # allocator map fresh blocks (a synchronous hipMalloc of GBs) every step. One send
        # buffer (forward sends, then the reverse exchange's receive), one received-halo
        # buffer per hidden layer (the last one is the reverse exchange's send after the
        # output layer's forward); the memory plan above counted exactly these
        self.send_buf, self.halo_buf = None, []
        self.ring_send, self.ring_recv = [], []
        self.aS_full = self.gz_full = None
        if graph.send_map is not None and not self.stream:
            self.send_buf = torch.empty(n_send, self.hid, **f)
            self.halo_buf = [torch.empty(H, self.hid, **f) for _ in range(self.nl - 1)]
        elif self.stream:
            # one arena: the ring's send / receive blocks, and (dead while the ring is idle,
            # in the output-layer backward) the sub-plan exchange's buffers
            blk_s, blk_r = n_send * self.cw, H * self.cw
            ring_fl = max(self.nbuf * (blk_s + blk_r), b.sub_bytes // 4)
            self.ring_arena = torch.empty(ring_fl, **f)
            ra = self.ring_arena
            self.ring_send = [ra[i * blk_s:(i + 1) * blk_s].view(n_send, self.cw)
                              for i in range(self.nbuf)]
            o = self.nbuf * blk_s
            self.ring_recv = [ra[o + i * blk_r:o + (i + 1) * blk_r].view(H, self.cw)
                              for i in range(self.nbuf)]
            self.agg_full = torch.empty(L, max(self.hid, self.d0), **f)
            self.aS_full = torch.empty(self.nS, self.w_lh, **f)
            # the reverse exchange's store: the output layer's aggregate store (dead after
            # the forward; stream-ordered on the compute stream like every use of both)
            self.gz_full = self.agg_full.view(-1)[:L * self.hid].view(L, self.hid) \
                if self.nl == 3 else None
        self.sub_hg = self.sub_sg = None
        if self.sub is not None:
            nh, nr = self.sub_rows
            if self.stream:
                self.sub_hg = self.ring_arena[:nh * self.hid].view(nh, self.hid)
                self.sub_sg = self.ring_arena[nh * self.hid:(nh + nr) * self.hid].view(
                    nr, self.hid)
            elif nh <= H and nr <= n_send:
                self.sub_hg = self.halo_buf[-1][:nh]
                self.sub_sg = self.send_buf[:nr]
        self.send_plan = self._send_plan(graph) \
            if (cfg.pack_fused and graph.send_map is not None and not self.stream) else None
        # the same for the pulled backward halo's rows of u (S-compacted rows)
        self._pull_send = None
        if self.send_plan is not None and self.pull is not None:
            rows = self.pull["send_rows"]
            ptr = torch.zeros(self.nS + 1, dtype=torch.long, device=dev)
            torch.cumsum(torch.bincount(rows, minlength=self.nS), 0, out=ptr[1:])
            self._pull_send = (ptr, torch.argsort(rows, stable=True).to(torch.int32)
                               .contiguous())
        if self.keep_as:
            self.aS_keep = self.aS_full if self.aS_full is not None else \
                torch.empty(self.nS, self.w_lh, **f)
        if self.store_sep:
            self.dZ = torch.empty(self.nS, self.hid, **f)
            self.u = torch.empty(self.nS, self.hid, **f) if self.nl == 3 else None
        else:
            hl = self.h[-1].view(-1)
            n = self.nS * self.hid
            self.dZ = hl[:n].view(self.nS, self.hid)
            self.u = hl[n:2 * n].view(self.nS, self.hid) if self.nl == 3 else None
        # ONE chunk arena: the aggregate and the logit / gradient chunk buffers during the
        # row-chunked passes, and the last hidden layer's keep bits (output-layer backward
        # only, when no chunk buffer is live)
        wA, wB = b.wA, b.wB
        bits_words = self.nS * (self.hid // 32)
        arena_fl = max(self.cr * (wA + wB), bits_words)
        self.arena = torch.empty(arena_fl, **f)
        self.bufA = self.arena[:self.cr * wA].view(self.cr, wA)
        self.bufB = self.arena[self.cr * wA:self.cr * (wA + wB)].view(self.cr, wB)
        self.bits = self.arena[:bits_words].view(torch.int32).view(self.nS, self.hid // 32)
        self.dz = torch.zeros(nT, self.Cg, **f)  # output-layer gradient rows
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
            elif dev.type != "cuda" or b.free - b.need_h > (4 * self.nS * self.hid + (8 << 30)):
                self.v_self = torch.empty(self.nS, self.hid, **f)
            # else: no room — the self term runs as a row-scattered GEMM per chunk
        self.acc_out_s = F32.WgradAcc(self.hid, self.Cg, dev)
        self.acc_out_n = F32.WgradAcc(self.hid, self.Cg, dev)
        kh = self.hid if self.nl == 3 else self.d0
        # (the bias gradients are the column sums of the same G: computed in the same
        # weight-gradient pass instead of separate column-sum passes)
        self.acc_hid_s = F32.WgradAcc(kh, self.hid, dev, colsum=True)
        self.acc_hid_n = F32.WgradAcc(kh, self.hid, dev)
        self.acc_in = F32.WgradAcc(2 * self.d0, self.hid, dev, colsum=True) \
            if self.nl == 3 else None

    def _agree(self, vals: List[int], op: str) -> List[int]:
        """``vals`` reduced elementwise (``"max"`` / ``"min"``) over the plan's group, so
        every rank takes the same branch; local values without peers (W=1, a rehearsal's
        loopback plan)."""
        import torch.distributed as dist

        g = self.g
        group = g.a2a.group if g.send_map is not None else None
        if not dist.is_initialized() or g.send_map is None or \
                dist.get_world_size(group) <= 1:
            return [int(v) for v in vals]
        from ..comm.groups import comm_device

        t = torch.tensor([int(v) for v in vals], dtype=torch.long, device=comm_device(group))
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.MIN,
                        group=group)
        return [int(v) for v in t.tolist()]

    def _aggT_setup(self) -> None:
        """Project-first output layer: the loss rows' aggregate of the last hidden layer
        (the operand of the W_neigh weight gradient) from a small CSR of the loss rows whose
        halo columns point at the rows pulled over the reversed output-layer sub-plan
        (the owners send the rows their peers' loss rows neighbour)."""
        dev, L, T = self.dev, self.L, self.T
        beg, end = self.adj.rp[T], self.adj.rp[T + 1]
        deg = end - beg
        nT = T.numel()
        rp = torch.zeros(nT + 1, dtype=torch.long, device=dev)
        torch.cumsum(deg, 0, out=rp[1:])
        nnz = int(rp[-1])
        pos = torch.repeat_interleave(beg - rp[:-1], deg, output_size=nnz) + \
            torch.arange(nnz, device=dev)
        col = self.adj.col[pos].long()
        del pos
        self._aggT_pull = None
        if self._sub_pull is not None:
            nz, recv_local, a2a_sub = self._sub_pull
            hm = torch.full((self.H,), -1, dtype=torch.long, device=dev)
            hm[nz.long()] = torch.arange(nz.numel(), device=dev)
            hal = col >= L
            col[hal] = L + hm[col[hal] - L]
            self._aggT_pull = (a2a_sub.reversed(), recv_local.long().contiguous(),
                               torch.empty(recv_local.numel(), self.hid,
                                           dtype=torch.float32, device=dev),
                               torch.empty(nz.numel(), self.hid, dtype=torch.float32,
                                           device=dev))
        bad = bool((col < 0).any())
        if bool(self._agree([int(bad)], "max")[0]):  # raised by every rank, or by none
            raise RuntimeError("FusedSAGE: a loss row neighbours a halo row outside the "
                               "output-layer sub-plan")
        self.aggT_rp, self.aggT_col = rp, col.to(torch.int32).contiguous()
        self.aggT = torch.empty(nT, self.hid, dtype=torch.float32, device=dev)

    def _aggT_issue(self, hl: torch.Tensor):
        """Send my rows of ``hl`` that the peers' loss rows neighbour (reversed sub-plan);
        returns the pending exchange or None."""
        if self._aggT_pull is None:
            return None
        a2a, rows, snd, rcv = self._aggT_pull
        K.copy_rows(hl, src_idx=rows, out=snd)
        return self._on_comm_stream(lambda: a2a(snd, out=rcv, async_op=True))

    def _aggT_finish(self, hl: torch.Tensor, pending) -> None:
        """``aggT = mean over the loss rows' neighbours of hl`` (local and pulled rows)."""
        kw = dict(row_scale=self.invdegT)
        if pending is not None:
            rcv, work = pending
            work.wait()
            kw.update(x2=rcv, nsplit=self.L)
        self._spmm(self.aggT_rp, self.aggT_col, hl, self.aggT, **kw)

    def _exchange_pf(self, Pb: torch.Tensor):
        """The projection's halo rows: packed into the (dead) send buffer, received into the
        last hidden layer's halo buffer (its rows are never exchanged in this mode)."""
        g, Cp = self.g, self.Cp
        snd = self.send_buf.view(-1)[:self.n_send * Cp].view(self.n_send, Cp)
        rcv = self.halo_buf[-1].view(-1)[:self.H * Cp].view(self.H, Cp)
        if self.send_plan is not None:  # packed by the projection GEMM
            return self._on_comm_stream(lambda: g.a2a(snd, out=rcv, async_op=True))
        if self.dev.type != "cuda":
            self._pack(Pb, "send", snd)
            return g.a2a(snd, out=rcv, async_op=True)
        self._pack(Pb, "send", snd)
        return self._on_comm_stream(lambda: g.a2a(snd, out=rcv, async_op=True))

    def _calibrate_link(self, g) -> float:
        """Per-peer rate of this job's halo all-to-all-v, measured once at setup (every rank
        of the plan's group calls it): 16 fp32 columns of every send row, twice, timed with
        stream events; the largest per-peer message over the slowest rank's time. The
        boundary-store planner (``_plan_store``) then weighs the exposed exchange against the
        transport this job actually gets (RCCL over xGMI on the node, the link model in a
        rehearsal) instead of the links' peak. ``cfg.plan_link_gbps`` > 0 (DGRAPH_PLAN_LINK_GBPS): that value."""
        if self.cfg.plan_link_gbps > 0:
            return self.cfg.plan_link_gbps
        if self.dev.type != "cuda":
            return PLAN_LINK_GBPS
        import torch.distributed as dist

        a2a, w = g.a2a, 16
        send = torch.zeros(a2a.total_send, w, dtype=torch.float32, device=self.dev)
        recv = torch.empty(a2a.total_recv, w, dtype=torch.float32, device=self.dev)
        a2a(send, out=recv)
        torch.cuda.synchronize(self.dev)
        peers = g._peers()
        if peers:
            dist.barrier(group=a2a.group)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(2):
            a2a(send, out=recv)
        e.record()
        torch.cuda.synchronize(self.dev)
        ms = torch.tensor([s.elapsed_time(e) / 2], dtype=torch.float64, device=self.dev)
        if peers:
            dist.all_reduce(ms, op=dist.ReduceOp.MAX, group=a2a.group)
        del send, recv
        peer = max(max(a2a.send_splits, default=0), max(a2a.recv_splits, default=0)) * w * 4
        t = float(ms) / 1e3
        return peer / t / 1e9 if peer > 0 and t > 0 else PLAN_LINK_GBPS

    def _pull_plan(self, g) -> dict:
        """The "pull" exchange of the input layer's backward (BWD_HALO): which of my send
        rows are in my S (their u rows travel) and which of my halo rows are in their
        owner's S (learned once through the forward plan: one exchange of a flag per send
        row), the sub-plan of the forward all-to-all-v restricted to those rows, the rows of
        u to pack, and one column map over local + halo columns: local c -> smap[c], halo
        L + h -> nS + (h's slot in the received rows), -1 where the source is not in S.
        The reference's halo backward is the push form: the received rows' gradient goes
        back through the reversed exchange and is scatter-added by the owners
        (DGraph/distributed/haloExchange.py:67-88); on a symmetric graph pulling the
        owners' nonzero gradient rows moves ~3.5x fewer bytes and needs no transposed pass
        over the halo."""
        dev, a2a = self.dev, g.a2a
        W = len(a2a.send_splits)
        sidx = g.send_map.idx.long()
        fs = self.smap[sidx] >= 0
        flag = fs.to(torch.float32).unsqueeze(1).expand(-1, 4).contiguous()  # 16-B rows
        fh = a2a(flag)[:, 0] > 0.5
        del flag
        peers = torch.arange(W, device=dev)
        ps = torch.repeat_interleave(peers, torch.tensor(a2a.send_splits, device=dev),
                                     output_size=sidx.numel())
        pr = torch.repeat_interleave(peers, torch.tensor(a2a.recv_splits, device=dev),
                                     output_size=fh.numel())
        cs = [int(v) for v in torch.bincount(ps[fs], minlength=W).tolist()]
        cr = [int(v) for v in torch.bincount(pr[fh], minlength=W).tolist()]
        del ps, pr
        n_recv = sum(cr)
        hm = torch.full((fh.numel(),), -1, dtype=torch.int32, device=dev)
        hm[fh] = torch.arange(n_recv, dtype=torch.int32, device=dev) + self.nS
        return {"a2a": AllToAllV(cs, cr, a2a.group),
                "send_rows": self.smap[sidx[fs]].long().contiguous(),
                "cmap": torch.cat([self.smap, hm]).contiguous(), "n_send": sum(cs),
                "n_recv": n_recv}

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

    @property
    def edges_aggregated(self) -> int:
        return self.g.edges_aggregated

    @edges_aggregated.setter
    def edges_aggregated(self, v: int) -> None:
        self.g.edges_aggregated = v

    @property
    def schedule(self) -> dict:
        """The overlap structure this executor runs (bench.py records it)."""
        return {"interior_rows": self.Li, "boundary_rows": self.L - self.Li,
                "chunk_rows": self.cr, "output_layer_store": self.agg_full is not None,
                "boundary_store": dict(self.use_store),
                "halo_stream": ({"column_block": self.cw, "buffers": self.nbuf}
                                if self.stream else False),
                "keep_agg0": self.agg0 is not None, "keep_aS": self.aS_keep is not None,
                "output_self_term_fill": self.zself is not None,
                "compact_T": self.TS is not None,
                "compact_halo_T": self.HTS is not None, "compact_pull": self.PT is not None,
                "support_rows": self.nS,
                "bwd_halo": "pull" if self.pull is not None else "push",
                "output_project_first": self.pf is not None,
                "memory_plan": list(self.memory_plan),
                **({"link_gbps_planned": round(self.link_gbps, 1)}
                   if self.g.send_map is not None else {})}

    # ------------------------------------------------------------------ helpers
    def _gemm(self, A1, B1, A2=None, B2=None, **kw):
        return F32.gemm_f32(A1, B1, A2, B2, **kw)

    def _spmm(self, rowptr, col, x, out=None, **kw):
        """fp32 SpMM at the column-pass width tuned for ``x``'s width (``_tune_passes``)."""
        kw.setdefault("pass_cols", self.pass_for.get(x.shape[1], 0))
        return F32.spmm_f32(rowptr, col, x, out, **kw)

    def _spmm_u(self, rowptr, col, u, out=None, **kw):
        """Column-mapped SpMM reading ``u``, a gradient stored on the support rows S only:
        full-width passes. The operand is ~S/L of a full activation, so one whole-row pass
        gathers about as many bytes per row window as a 64-column pass over full rows, and
        the entries and their column map are walked once instead of once per pass:
        column-mapped F=256 at 30 % of rows 48.9 -> 30.2 ms (64- vs 256-column passes),
        the W=1 step 1959 -> 1867 ms. Over an S-compacted adjacency (``TS``/``HTS``, no map
        to walk) the tuned narrow passes stay faster (W=8 265.6 vs 271.1 ms)."""
        forced = self.cfg.pass_cols
        w = u.shape[1]
        if forced:
            pc = min(forced, w)
        else:
            # full width only while u is a small share of the rows: on ogbn-products
            # (support ~ most rows) full-width passes lose (bwd_l0 21.3 vs 17.0 ms)
            base = self.pass_for.get(w, 0)
            frac = self.nS / max(self.L, 1)
            pc = min(w, 256) if (not base or base >= w or frac <= self.cfg.u_full_frac) else base
        kw.setdefault("pass_cols", pc)
        return F32.spmm_f32(rowptr, col, u, out, **kw)

    def _agg(self, hin: torch.Tensor, r0: int, r1: int, out: torch.Tensor, part: str = "all",
             halo: Optional[torch.Tensor] = None, **kw) -> torch.Tensor:
        """``out = mean over in-neighbours`` of rows [r0, r1), ``part`` of each row's entries
        ("all" / "int" / "halo"); halo columns read ``halo`` (received rows). "all" without
        ``halo`` is only valid for rows that have no halo entry."""
        rp, re = self.adj.rows(r0, r1, part)
        if part != "int" and halo is not None and self.adj.mid is not None:
            kw.update(x2=halo, nsplit=self.L)
        kw.setdefault("row_scale", self.inv_deg[r0:r1])
        return self._spmm(rp, self.adj.col, hin, out, rowend=re, **kw)

    def _tune_passes(self) -> None:
        """Column-pass width per operand width, from the graph's locality: on a graph whose
        neighbour lists stay near the row (most entries within +-2^16 ids), narrow
        (64-column) passes keep each pass's window of neighbour rows in the L2 / Infinity
        Cache (13.1 TB/s effective vs 9.8 at 128 columns on the bench graph); on a graph
        without that locality every neighbour row is a random HBM access and full-width
        passes read each row once, in one burst, instead of once per pass (structureless
        papers100M step 5508 -> 3687 ms, profiles/r03/). The locality is
        parallel/reorder.graph_locality of the graph's ORIGINAL order (a rank renumbered
        interior-first carries it as ``locality_hint``). DGRAPH_FUSED_PASS_COLS forces a
        width."""
        self.pass_for = {}
        forced = self.cfg.pass_cols
        if forced:
            self.pass_for = {self.d0: min(forced, self.d0), self.hid: min(forced, self.hid)}
            return
        if self.dev.type != "cuda" or self.locality is None:
            return
        for w in (self.d0, self.hid):
            self.pass_for[w] = 64 if self.locality >= 0.5 else w

    @staticmethod
    def _csr_range(csr, r0: int, r1: int):
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

    def _send_plan(self, g):
        """The fused pack's plan: local row r's positions in the forward send buffer are
        ``pos[ptr[r]:ptr[r + 1]]`` (a row sent to several peers has several). Replaces the
        gather of the send rows before each all-to-all-v (the reference packs per exchange,
        DGraph/distributed/haloExchange.py:47-62)."""
        sidx = g.send_map.idx.long()
        order = torch.argsort(sidx, stable=True)
        ptr = torch.zeros(self.L + 1, dtype=torch.long, device=self.dev)
        torch.cumsum(torch.bincount(sidx, minlength=self.L), 0, out=ptr[1:])
        if int(ptr[-1]) != self.n_send:
            raise RuntimeError("FusedSAGE: send rows outside the local rows")
        return ptr, order.to(torch.int32).contiguous()

    def _send_arg(self, r0: int, r1: int, width: int):
        """``send=`` of the GEMM producing rows [r0, r1) of an exchanged activation (None
        when no fused pack or no sent row in the range)."""
        if self.send_plan is None or r1 <= self.Li:
            return None
        ptr, pos = self.send_plan
        snd = self.send_buf.view(-1)[:self.n_send * width].view(self.n_send, width)
        return snd, ptr[r0:r1 + 1], pos

    def _pack(self, x: torch.Tensor, which: str, out: torch.Tensor) -> None:
        """``out[i] = x[src[i]]`` for the send rows of the forward plan (``which`` =
        "send") or of the pulled backward halo ("pull"), issued in SOURCE-row order: a row
        sent to k peers is read k times back to back (the repeats hit the cache) instead of
        k times far apart, and written to its k send-buffer positions. Each pack of a
        structureless W=8 rank read ~3.5x its unique rows from HBM (the pack was 78 ms of a
        565 ms step, profiles/r06/structureless_w8_rank_kernels_per_step.txt)."""
        p = self._packs.get(which)
        if p is None:
            src = (self.g.send_map.idx if which == "send" else self.pull["send_rows"]).long()
            order = torch.argsort(src, stable=True)
            idt = torch.int32 if max(src.numel(), int(src.max()) + 1 if src.numel() else 0) \
                < 2 ** 31 else torch.long
            p = (src[order].to(idt).contiguous(), order.to(idt).contiguous())
            self._packs[which] = p
        K.copy_rows(x, src_idx=p[0], dst_idx=p[1], out=out)

    def _exchange(self, h: torch.Tensor, l: int):
        """Start the halo rows of hidden layer ``l``'s output ``h`` on their way from their
        owners (forward all-to-all-v, asynchronous, resident buffers): ``(recv, work)``, or
        None at W=1. With the fused pack the send buffer was filled by h's GEMMs."""
        g = self.g
        if g.send_map is None:
            return None
        if self.send_plan is not None:
            return self._on_comm_stream(
                lambda: g.a2a(self.send_buf, out=self.halo_buf[l], async_op=True))
        if self.dev.type != "cuda":
            self._pack(h, "send", self.send_buf)
            return g.a2a(self.send_buf, out=self.halo_buf[l], async_op=True)
        # pack and send on the communication stream: the pack (a streaming gather of the
        # send rows) overlaps the next layer's interior work instead of preceding it. It
        # reads h (complete: the stream waits for the compute stream) and writes the send
        # buffer, whose previous exchange the compute stream has already waited for
        if self.cfg.pack_stream == "compute":
            self._pack(h, "send", self.send_buf)
            return self._on_comm_stream(
                lambda: g.a2a(self.send_buf, out=self.halo_buf[l], async_op=True))
        from ..comm.alltoallv import _side_stream

        side = _side_stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            self._pack(h, "send", self.send_buf)
            return g.a2a(self.send_buf, out=self.halo_buf[l], async_op=True)

    def _plan_store(self) -> dict:
        """Per forward layer (by output width): pre-aggregate the boundary rows' interior
        part while the exchange is in flight? Only when the exchange the interior rows
        leave exposed — the modelled transfer (largest per-peer message / PLAN_LINK_GBPS)
        minus the interior rows' work (SpMM bytes and GEMM flops at the planning rates) —
        exceeds twice what the store costs (a read-modify-write of every boundary row's
        aggregate): at W=2 on the bench graph the store cost more than the ~6 ms it hid
        and its output-layer buffer displaced the kept input aggregate (a 973 ms rank step
        without, 1022 ms with, profiles/r05/)."""
        g = self.g
        mode = self.cfg.boundary_store
        if mode in ("on", "off") or g.send_map is None or self.Li >= self.L:
            return {k: mode == "on" for k in ("hidden", "out")}
        a2a = g.a2a
        peer_rows = max(max(a2a.send_splits, default=0), max(a2a.recv_splits, default=0))
        t_x = peer_rows * self.hid * 4 / (self.link_gbps * 1e9)
        nnz_a = int(self.adj.rp[self.Li]) if self.Li > 0 else 0
        t_store = 2.0 * (self.L - self.Li) * self.hid * 4 / (PLAN_HBM_TBPS * 1e12)
        out = {}
        for key, n_out in (("hidden", self.hid), ("out", self.Cp)):
            t_a = nnz_a * self.hid * 4 / (PLAN_SPMM_TBPS * 1e12) + \
                2.0 * self.Li * 2 * self.hid * n_out / (PLAN_GEMM_TFPS * 1e12)
            out[key] = t_x - t_a > 2.0 * t_store
        return out

    def _layer(self, hin: torch.Tensor, halo, consume, width: int, name: str,
               store: Optional[torch.Tensor] = None, keep: Optional[torch.Tensor] = None):
        """Aggregate every row chunk of ``hin`` and hand it to ``consume(ci, agg)``.
        ``halo``: None (W=1), the received (resident) halo rows, or a pending
        ``(recv, work)`` exchange. Resident / none: one pass per chunk. Pending: the
        interior chunks [0, Li) first (they need no halo row); then, with a ``store``
        ([>= L - Li, >= width] rows free until the consumer writes boundary row r, e.g.
        the layer's own output buffer — the GEMM of a chunk reads its aggregate rows before
        it overwrites them, tile by tile), the interior part of every boundary row; then
        the exchange is waited for and the boundary chunks finish (halo part into the
        store, or one pass). ``keep`` ([L, width]): aggregate there instead of the chunk
        buffer (kept after the step). Returns the halo rows (for the backward)."""
        items = [ci for ci, (r0, r1) in enumerate(self.chunks) if r1 > r0]
        pending = isinstance(halo, tuple)

        def buf(ci):
            r0, r1 = self.chunks[ci]
            return keep[r0:r1, :width] if keep is not None else self.bufA[:r1 - r0, :width]

        if not pending:
            for ci in items:
                r0, r1 = self.chunks[ci]
                consume(ci, self._agg(hin, r0, r1, buf(ci), "all", halo))
            return halo
        recv, work = halo
        seg_a = [ci for ci in items if ci < self.nA]
        seg_b = [ci for ci in items if ci >= self.nA]
        if not self.cfg.overlap:
            self._mark(f"exchange_{name}")
            work.wait()
            self._mark(name)
            for ci in items:
                r0, r1 = self.chunks[ci]
                consume(ci, self._agg(hin, r0, r1, buf(ci), "all", recv))
            return recv
        for ci in seg_a:
            r0, r1 = self.chunks[ci]
            consume(ci, self._agg(hin, r0, r1, buf(ci), "all"))
        Li = self.Li
        if store is not None and keep is None:
            for ci in seg_b:
                r0, r1 = self.chunks[ci]
                self._agg(hin, r0, r1, store[r0 - Li:r1 - Li, :width], "int")
        else:
            store = None
        self._mark(f"exchange_{name}")
        work.wait()
        self._mark(name)
        for ci in seg_b:
            r0, r1 = self.chunks[ci]
            if store is not None:
                a = store[r0 - Li:r1 - Li, :width]
                self._agg(hin, r0, r1, a, "halo", recv, beta=1.0)
            else:
                a = self._agg(hin, r0, r1, buf(ci), "all", recv)
            consume(ci, a)
        return recv

    def _on_comm_stream(self, fn):
        """Run ``fn()`` (a pack + an asynchronous exchange) on the communication stream,
        behind the compute stream's work so far (CPU: inline)."""
        if self.dev.type != "cuda":
            return fn()
        from ..comm.alltoallv import _side_stream

        side = _side_stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            return fn()

    def _stream_blocks(self, F: int) -> List[Tuple[int, int]]:
        """Column blocks of a streamed exchange of width ``F``: ``cw`` wide, the first one
        ``cw / 2`` (STREAM_RAMP) so the pipeline fill is short."""
        cw = self.cw
        if self.cfg.stream_ramp and cw >= 64 and F > cw:
            return [(0, cw // 2)] + _ranges(cw // 2, F, cw)
        return _ranges(0, F, cw)

    @staticmethod
    def _ring(bufs, b: int, w: int) -> torch.Tensor:
        """Ring buffer ``b`` as a contiguous ``[rows, w]`` block (w <= its width)."""
        t = bufs[b]
        return t if t.shape[1] == w else t.view(-1)[:t.shape[0] * w].view(t.shape[0], w)

    def _stream_fwd(self, h: torch.Tensor, out: torch.Tensor, name: str,
                    rows: Optional[torch.Tensor] = None, fill=None) -> None:
        """Streamed halo: ``out[:, c] = mean over in-neighbours of h[:, c]`` for every row
        (or for the adjacency rows ``rows``, output row i <- rows[i]), with h's halo rows
        exchanged in column blocks of ``cw`` through the buffer ring — block k+1 is on the
        links while block k is aggregated (two-source: local and received rows in one
        pass). A block's buffers are reused only after the compute stream consumed them
        (the comm stream waits for it before every pack)."""
        g, L, nb = self.g, self.L, self.nbuf
        blocks = self._stream_blocks(h.shape[1])

        def issue(k):
            c0, c1 = blocks[k]
            b = k % nb
            snd = self._ring(self.ring_send, b, c1 - c0)
            rcv = self._ring(self.ring_recv, b, c1 - c0)

            if self.cfg.pack_stream == "compute":
                self._pack(h[:, c0:c1], "send", snd)
                return self._on_comm_stream(lambda: g.a2a(snd, out=rcv, async_op=True))

            def go():
                self._pack(h[:, c0:c1], "send", snd)
                return g.a2a(snd, out=rcv, async_op=True)
            return self._on_comm_stream(go)

        works = {0: issue(0)}
        for k, (c0, c1) in enumerate(blocks):
            if nb > 1 and k + 1 < len(blocks):
                works[k + 1] = issue(k + 1)
            if k == 0 and fill is not None:
                fill()  # independent compute-stream work while block 0 is on the links
            recv, work = works.pop(k)
            self._mark(f"exchange_{name}")
            work.wait()
            self._mark(name)
            if rows is None:
                self._spmm(self.adj.rp, self.adj.col, h[:, c0:c1], out[:, c0:c1], x2=recv,
                           nsplit=L, row_scale=self.inv_deg, pass_cols=c1 - c0)
            else:
                self._spmm(self.adj.rp, self.adj.col, h[:, c0:c1], out[:, c0:c1],
                           row_ids=rows, x2=recv, nsplit=L, row_scale=self.invdegS,
                           pass_cols=c1 - c0)
            if nb == 1 and k + 1 < len(blocks):
                works[k + 1] = issue(k + 1)

    def _stream_rev(self, u: torch.Tensor, gz: torch.Tensor, gate: torch.Tensor,
                    name: str, fill=None) -> None:
        """Streamed reverse exchange of B1b: for every column block, the halo rows'
        contributions ``A_halo^T u`` (column-mapped onto S) are sent to their owners and
        summed into ``gz`` (zeroed first; the ReLU gate of layer 0 applied), block k+1's
        contributions computed while block k is on the links."""
        g, nb = self.g, self.nbuf
        blocks = self._stream_blocks(u.shape[1])
        gz.zero_()
        st = self.send_st

        def issue(k):
            c0, c1 = blocks[k]
            b = k % nb
            hg = self._ring(self.ring_recv, b, c1 - c0)
            snd = self._ring(self.ring_send, b, c1 - c0)
            if self.HTS is not None:
                self._spmm(self.HTS[0], self.HTS[1], u[:, c0:c1], hg)
            else:
                self._spmm_u(self.haloT.rowptr, self.haloT.col, u[:, c0:c1], hg,
                             col_map=self.smap)
            return self._on_comm_stream(lambda: g.a2a_rev(hg, out=snd, async_op=True))

        works = {0: issue(0)}
        for k, (c0, c1) in enumerate(blocks):
            if nb > 1 and k + 1 < len(blocks):
                works[k + 1] = issue(k + 1)
            if k == 0 and fill is not None:
                fill()
            sg, work = works.pop(k)
            self._mark(f"exchange_{name}")
            work.wait()
            self._mark(name)
            self._spmm(st.rowptr, st.col, sg, gz[:, c0:c1], beta=1.0, row_map=st.row_map,
                       gate=gate[:, c0:c1])
            if nb == 1 and k + 1 < len(blocks):
                works[k + 1] = issue(k + 1)

    def _stream_pull(self, u: torch.Tensor, v: Optional[torch.Tensor], gz: torch.Tensor,
                     gate: torch.Tensor, name: str, fill=None) -> None:
        """Streamed pull of B1b: for every column block, my S rows of u that are halo rows
        elsewhere are packed and sent (the pull sub-plan), and once block k has landed
        ``gz[:, c] = gate(sum over the row's local and halo support neighbours of u[:, c]
        + v[:, c])`` for every row in one column-mapped two-source pass, block k+1 on the
        links meanwhile."""
        pl, nb = self.pull, self.nbuf
        blocks = self._stream_blocks(u.shape[1])

        def rows(bufs, b, n, w):
            return bufs[b].view(-1)[:n * w].view(n, w)

        def issue(k):
            c0, c1 = blocks[k]
            b = k % nb
            snd = rows(self.ring_send, b, pl["n_send"], c1 - c0)
            rcv = rows(self.ring_recv, b, pl["n_recv"], c1 - c0)
            self._pack(u[:, c0:c1], "pull", snd)
            return self._on_comm_stream(lambda: pl["a2a"](snd, out=rcv, async_op=True))

        works = {0: issue(0)}
        for k, (c0, c1) in enumerate(blocks):
            if nb > 1 and k + 1 < len(blocks):
                works[k + 1] = issue(k + 1)
            if k == 0 and fill is not None:
                fill()
            uh, work = works.pop(k)
            self._mark(f"exchange_{name}")
            work.wait()
            self._mark(name)
            sa = {} if v is None else dict(self_add=v[:, c0:c1], self_map=self.smap)
            if self.PT is not None:
                self._spmm(self.PT[0], self.PT[1], u[:, c0:c1], gz[:, c0:c1], x2=uh,
                           nsplit=self.nS, gate=gate[:, c0:c1], pass_cols=c1 - c0, **sa)
            else:
                self._spmm_u(self.adj.rp, self.adj.col, u[:, c0:c1], gz[:, c0:c1],
                             col_map=pl["cmap"], x2=uh, nsplit=self.nS, gate=gate[:, c0:c1],
                             pass_cols=c1 - c0, **sa)
            if nb == 1 and k + 1 < len(blocks):
                works[k + 1] = issue(k + 1)

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
        self._mark("fwd_l0")
        nnz = self.nnz_it + self.nnz_h
        # ---------------- forward: hidden layers
        hin, hin_halo = x, (g._static_halo(x) if g.send_map is not None else None)
        halos = []
        for l in range(nl - 1):
            ws, wn, b = P[l]
            if l == 0:
                ws, wn = self._pad_in(ws), self._pad_in(wn)
            else:
                ws, wn = ws.detach().contiguous(), wn.detach().contiguous()
            hout = self.h[l]
            bias = b.detach()

            keep_s = self.aS_keep if l == nl - 2 else None

            # (this layer's output is exchanged next unless the projected output layer
            # exchanges its projection instead)
            sends = not self.stream and not (self.pf is not None and l == nl - 2)

            def consume(ci, a, hin=hin, hout=hout, ws=ws, wn=wn, bias=bias, keep_s=keep_s,
                        sends=sends):
                r0, r1 = self.chunks[ci]
                if keep_s is not None:
                    self._keep_s_rows(ci, a, keep_s)
                self._gemm(hin[r0:r1], ws, a, wn, bias=bias, relu=True, out=hout[r0:r1],
                           send=self._send_arg(r0, r1, hout.shape[1]) if sends else None)

            if self.stream and l > 0 and not self.cfg.stream_fill:
                self._stream_fwd(hin, hout, f"fwd_l{l}")
                for ci, (r0, r1) in enumerate(self.chunks):
                    if r1 > r0:
                        consume(ci, hout[r0:r1])
                halos.append(None)
            elif self.stream and l > 0:
                # streamed halo: every row's aggregate into the output layer's store
                # (column block by column block; free until the output layer), while the
                # self term h W_self + b runs into the layer's output buffer during the
                # first block's transfer (the pipeline fill); then per chunk
                # h_out = relu(agg W_neigh + h_out)
                agg = self.agg_full[:, :hin.shape[1]]
                self._stream_fwd(hin, agg, f"fwd_l{l}",
                                 fill=lambda hin=hin, ws=ws, bias=bias, hout=hout:
                                 self._gemm(hin, ws, bias=bias, out=hout))
                for ci, (r0, r1) in enumerate(self.chunks):
                    if r1 > r0:
                        a = agg[r0:r1]
                        if keep_s is not None:
                            self._keep_s_rows(ci, a, keep_s)
                        self._gemm(a, wn, cin=hout[r0:r1], beta=1.0, relu=True,
                                   out=hout[r0:r1])
                halos.append(None)
            else:
                # layer l >= 1 can store boundary-row aggregates in its own output buffer
                store = hout[self.Li:] if (l > 0 and hin.shape[1] == hout.shape[1] and
                                           self.use_store["hidden"]) else None
                keep = self.agg0 if l == 0 else None
                halos.append(self._layer(hin, hin_halo, consume, hin.shape[1], f"fwd_l{l}",
                                         store=store, keep=keep))
            self.edges_aggregated += nnz
            hin = hout
            # this layer's halo rows leave now and land while the next layer works
            hin_halo = None if (self.stream or (self.pf is not None and l == nl - 2)) \
                else self._exchange(hout, l)
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
        if self.pf is not None:
            # project first: Pb = h W_neigh (send rows first, so the exchange leaves while
            # the interior rows are projected), then the logits of every row chunk
            # z = h W_self + b + mean_N(Pb); the loss rows' aggregate of h (for the W_neigh
            # weight gradient) from the pulled rows, at the end
            Pb, Li = self.pf, self.Li
            tw = self._aggT_issue(hl)
            self._gemm(hl[Li:], wnp, out=Pb[Li:],
                       send=None if self.stream else self._send_arg(Li, self.L, Cp))
            out_pf = lambda ci, a: self._out_chunk(ci, a, hl, wsp, wnp, bp, pf=True)  # noqa
            if self.stream:
                self._stream_fwd(Pb, self.agg_full[:, :Cp], "fwd_out",
                                 fill=(lambda: self._gemm(hl[:Li], wnp, out=Pb[:Li]))
                                 if Li > 0 else None)
                for ci, (r0, r1) in enumerate(self.chunks):
                    if r1 > r0:
                        out_pf(ci, self.agg_full[r0:r1, :Cp])
                hl_halo = None
            else:
                pend = self._exchange_pf(Pb)
                if Li > 0:
                    self._gemm(hl[:Li], wnp, out=Pb[:Li])
                hl_halo = self._layer(Pb, pend, out_pf, Cp, "fwd_out",
                                      store=self.agg_full if self.use_store["out"] else None)
            self._aggT_finish(hl, tw)
        elif self.stream:
            zs = self.zself
            self._stream_fwd(hl, self.agg_full, "fwd_out",
                             fill=None if zs is None else
                             (lambda: self._gemm(hl, wsp, bias=bp, out=zs)))
            for ci, (r0, r1) in enumerate(self.chunks):
                if r1 > r0:
                    self._out_chunk(ci, self.agg_full[r0:r1, :hid], hl, wsp, wnp, bp)
            hl_halo = None
        else:
            hl_halo = self._layer(hl, hin_halo, lambda ci, a: self._out_chunk(ci, a, hl, wsp,
                                                                              wnp, bp),
                                  hid, "fwd_out",
                                  store=self.agg_full if self.use_store["out"] else None)
        halos.append(hl_halo)
        self.edges_aggregated += nnz
        # per-row losses / hits summed once, in a fixed order
        loss = self.row_loss.sum() * self.inv_n
        hv = self.hit.long()
        self.correct[0] = (hv * self.E_val_l).sum()
        self.correct[1] = (hv * (1 - self.E_val_l)).sum()
        self._mark("bwd_out")
        return self._backward(P, halos, hl, hl_halo, loss)

    def _keep_s_rows(self, ci, a, keep):
        """The support rows of chunk ci's aggregate ``a`` into ``keep`` (rows in S order),
        before the chunk's GEMM consumes (or, in place, overwrites) it."""
        s0, s1 = self.ch_S[ci]
        if s1 > s0:
            K.copy_rows(a, src_idx=self.ch_Sloc[ci], out=keep[s0:s1])

    def _out_chunk(self, ci, a, hl, wsp, wnp, bp, pf: bool = False):
        """Output layer of row chunk ci: logits of every row, the loss rows' cross-entropy
        gradient and output-layer weight gradients, eval hits. ``pf``: ``a`` is the chunk's
        aggregate of the projection h W_neigh (project-first), not of h."""
        C, Cp = self.C, self.Cp
        r0, r1 = self.chunks[ci]
        n = r1 - r0
        if pf:
            z = self._gemm(hl[r0:r1], wsp, bias=bp, cin=a, beta=1.0, out=self.bufB[:n, :Cp])
        elif self.stream and self.zself is not None:  # self term from the pipeline fill
            z = self._gemm(a, wnp, cin=self.zself[r0:r1], beta=1.0, out=self.bufB[:n, :Cp])
        else:
            z = self._gemm(hl[r0:r1], wsp, a, wnp, bias=bp, out=self.bufB[:n, :Cp])
        t0, t1 = self.ch_T[ci]
        if t1 > t0:
            # one fused kernel: per-row loss and the scaled softmax gradient rows
            tl = self.ch_Tloc[ci]
            dzt = self.dz[t0:t1]
            F32.xent_rows(z, tl, self.yT[t0:t1], self.inv_n, dzt, self.row_loss[t0:t1], C)
            # (the self-term weight gradient h[T]^T dz runs once over all loss rows in the
            # backward; the aggregate rows a[T] exist only per chunk)
            if not pf:
                self.acc_out_n.add(a, dzt, a1_rows=tl)
        e0, e1 = self.ch_E[ci]
        if e1 > e0:
            F32.argmax_hits(z, self.ch_Eloc[ci], self.yE[e0:e1], self.hit[e0:e1], C)

    def _backward(self, P, halos, hl, hl_halo, loss):
        g, x, dev = self.g, self.x, self.dev
        nl, hid, C, Cg = self.nl, self.hid, self.C, self.Cg
        ws, wn, _ = P[nl - 1]
        # ---------------- backward: output layer -> dZ of the last hidden layer on S
        hlast = hl
        F32.row_keep_bits(hlast, self.S, self.bits)  # the last hidden ReLU derivative on S
        del hl_halo, halos[-1]
        gw = {}
        self.acc_out_s.add(hlast, self.dz, a1_rows=self.T)  # one call over every loss row
        if self.pf is not None:  # project-first: the loss rows' aggregate of h, pulled
            self.acc_out_n.add(self.aggT, self.dz)
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
            hg = self._spmm(ht_nz.rowptr, ht_nz.col, u2, self.sub_hg)
            sg, work = a2a_sub(hg, out=self.sub_sg, async_op=True)
            self.edges_aggregated += ht_nz.nnz
        # the last hidden layer's ReLU derivative applied by each writer of dZ (a 0/1 mask
        # distributes over the sum): the aggregations in their epilogue from the keep bits,
        # the loss rows' self term afterwards on those rows only — instead of a pass that
        # re-reads and re-writes all of dZ
        self._spmm(self.AT_S.rowptr, self.AT_S.col, u2, dZ, keep_bits=self.bits)
        self.edges_aggregated += self.AT_S.nnz
        if work is not None:
            self._mark("exchange_bwd_out")
            work.wait()
            self._mark("bwd_out")
            self._spmm(stc.rowptr, stc.col, sg, dZ, beta=1.0, row_map=stc_rows,
                       keep_bits=self.bits)
            del sg, hg
        self._gemm(self.dz, ws_t, cin=dZ, o_rows=self.posT, out=dZ)
        F32.apply_keep_bits(dZ, self.bits, rows=self.posT)
        # ---------------- backward: last hidden layer (index nl-2) weights over S rows
        lh = nl - 2
        self._mark(f"bwd_l{lh}")
        ws1, wn1, _ = P[lh]
        hin_l = x if lh == 0 else self.h[lh - 1]
        hin_l_halo = halos[lh]
        u = None
        work = None
        self.acc_hid_s.reset()
        self.acc_hid_n.reset()
        halo_l = hin_l_halo if self.adj.mid is not None else None
        kept = self.aS_keep is not None
        streamed = self.stream and lh > 0 and not kept

        def s_rows():
            """The last hidden layer's weight gradients over the S rows."""
            if streamed:
                # the S rows' aggregate of h1, its halo rows re-fetched in column blocks
                self._stream_fwd(hin_l, self.aS_full, f"bwd_l{lh}", rows=self.S)
            for s0, s1 in self.s_chunks:
                if s1 <= s0:
                    continue
                rows = self.S[s0:s1]
                if kept:  # from the forward: no second aggregation of the S rows
                    aS = self.aS_keep[s0:s1]
                elif streamed:
                    aS = self.aS_full[s0:s1]
                else:
                    aS = self.bufA[:s1 - s0, :hin_l.shape[1]]
                    kw = dict(x2=halo_l, nsplit=self.L) if halo_l is not None else {}
                    self._spmm(self.adj.rp, self.adj.col, hin_l, aS, row_ids=rows,
                               row_scale=self.invdegS[s0:s1], **kw)
                self.acc_hid_s.add(hin_l, dZ[s0:s1], a1_rows=rows)
                self.acc_hid_n.add(aS, dZ[s0:s1])
            if not kept:
                self.edges_aggregated += self.nnz_S

        pending_s = True
        uh, v_pre, full = None, None, False
        if nl == 3:
            # u1 = (dZ1 Wn1^T) / deg_S: its transposed aggregation feeds layer 0; the halo
            # part is computed and sent first so the exchange overlaps the S-row work and
            # the interior rows of layer 0 below
            pull_res = self.pull is not None and not self.stream
            if pull_res:
                pl = self.pull
                snd = self.send_buf.view(-1)[:pl["n_send"] * hid].view(pl["n_send"], hid)
                rcv = self.halo_buf[-1].view(-1)[:pl["n_recv"] * hid].view(pl["n_recv"], hid)
            # (pulled, resident: the pack of u's sent rows fused into u's GEMM)
            u = self._gemm(dZ, wn1.detach().t().contiguous(), row_scale=self.invdegS,
                           out=self.u,
                           send=(snd, *self._pull_send) if (pull_res and self._pull_send)
                           else None)
            if pull_res:
                # pull: my S rows of u that are halo rows elsewhere leave now (packed into
                # the dead forward send buffer; received into the output layer's dead halo
                # buffer) and land while the S-row work and layer 0's interior rows run
                if not self._pull_send:
                    self._pack(u, "pull", snd)
                uh, work = self._on_comm_stream(
                    lambda: pl["a2a"](snd, out=rcv, async_op=True))
            elif self.pull is not None:
                # streamed pull: u's column blocks (my S rows that are halo rows elsewhere)
                # through the buffer ring, every row of the input-layer gradient aggregated
                # block by block into its store — local and received rows in one pass, the
                # support rows' self term and layer 0's ReLU gate in its epilogue; the S-row
                # weight gradients (aggregate kept from the forward) fill the first transfer
                ws1_t = P[1][0].detach().t().contiguous()
                v_pre = self._gemm(dZ, ws1_t, out=self.v_self) \
                    if self.v_self is not None else None
                self._stream_pull(u, v_pre, self.gz_full, self.h[0], f"bwd_l{lh}",
                                  fill=s_rows if kept else None)
                pending_s = not kept
                full = True
            elif self.haloT is not None and self.stream:
                # streamed reverse exchange into the input-layer gradient store; with the
                # S-row aggregate kept from the forward, the S-row weight gradients need
                # nothing from it and fill the pipeline's first transfer
                self._stream_rev(u, self.gz_full, self.h[0], f"bwd_l{lh}",
                                 fill=s_rows if kept else None)
                pending_s = not kept
                self.edges_aggregated += self.haloT.nnz
            elif self.haloT is not None:
                # the output layer's received halo rows are dead: its buffer sends, the
                # forward send buffer receives
                if self.HTS is not None:
                    hg1 = self._spmm(self.HTS[0], self.HTS[1], u, self.halo_buf[-1])
                else:
                    hg1 = self._spmm_u(self.haloT.rowptr, self.haloT.col, u, self.halo_buf[-1],
                                       col_map=self.smap)
                sg1, work = g.a2a_rev(hg1, out=self.send_buf, async_op=True)
                self.edges_aggregated += self.haloT.nnz
        if pending_s:
            s_rows()
        gw[(lh, 0)] = self.acc_hid_s.result()
        gw[(lh, 1)] = self.acc_hid_n.result()
        gw[(lh, 2)] = self.acc_hid_s.col_result()
        if lh == 0:
            gw[(0, 0)], gw[(0, 1)] = gw[(0, 0)][:self.d0_in], gw[(0, 1)][:self.d0_in]
        if nl == 3:
            self._input_layer_backward(P, halos, dZ, u, work,
                                       sg1 if (work is not None and uh is None) else None,
                                       gw, uh, full, v_pre)
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

    def _input_layer_backward(self, P, halos, dZ, u, work, sg1, gw, uh=None, full=False,
                              v=None):
        """B1b: dZ0 by row chunks, consumed at once by the input layer's weight gradients.
        Interior chunks (no row receives from the reverse exchange) run before it is
        waited for. ``uh``: the received S rows of u of the "pull" exchange (the boundary
        chunks aggregate local and halo entries in one pass). ``full``: the streamed pull
        left every row's finished gradient (self term ``v`` and gate applied) in the
        store."""
        x, dev, hid = self.x, self.dev, self.hid
        ws1 = P[1][0]
        ws1_t = ws1.detach().t().contiguous()
        self._mark("bwd_l0")
        self.acc_in.reset()
        h1 = self.h[0]
        x_halo = halos[0] if self.adj.mid is not None else None
        # the support rows' own term dZ1 Ws1^T, once over S (one full-size GEMM instead
        # of a row-scattered one per chunk); added by the aggregation's epilogue
        if not full:
            v = self._gemm(dZ, ws1_t, out=self.v_self) if self.v_self is not None else None
        items = [ci for ci, (r0, r1) in enumerate(self.chunks) if r1 > r0]
        waited = work is None
        for ci in items:
            r0, r1 = self.chunks[ci]
            n = r1 - r0
            if not waited and ci >= self.nA:
                self._mark("exchange_bwd_l0")
                work.wait()
                waited = True
                self._mark("bwd_l0")
            # memory-bound: the column-mapped transposed aggregation of u1 (gated by layer
            # 0's ReLU) and the layer-0 input aggregate (kept from the forward or recomputed)
            sa = dict(gate=h1[r0:r1], self_add=v, self_map=self.smap if v is not None else None,
                      self_row0=r0)
            if full:
                gz = self.gz_full[r0:r1]
            elif self.gz_full is not None:
                # streamed reverse exchange (already gated): the aggregation accumulates
                # into its rows in place (beta = 1; gate(old + new) = old + gate(new) for
                # a gated old) instead of an elementwise add pass per chunk
                gz = self.gz_full[r0:r1]
                sa["beta"] = 1.0
            else:
                gz = self.bufB[:n, :hid]
            if full:
                pass
            elif uh is not None and ci >= self.nA and self.PT is not None:
                self._spmm(self.PT[0][r0:r1 + 1], self.PT[1], u, gz, x2=uh, nsplit=self.nS,
                           **sa)
            elif uh is not None and ci >= self.nA:
                rp, _ = self.adj.rows(r0, r1, "all")
                self._spmm_u(rp, self.adj.col, u, gz, col_map=self.pull["cmap"], x2=uh,
                             nsplit=self.nS, **sa)
            elif self.TS is not None:
                self._spmm(self.TS[0][r0:r1 + 1], self.TS[1], u, gz, **sa)
            elif self.itT is not None:
                self._spmm_u(self.itT.rowptr[r0:r1 + 1], self.itT.col, u, gz,
                             col_map=self.smap, **sa)
            else:
                rp, re = self.adj.rows(r0, r1, "int")
                self._spmm_u(rp, self.adj.col, u, gz, rowend=re, col_map=self.smap, **sa)
            sr = self.ch_send[ci]
            if self.gz_full is None and sg1 is not None and sr is not None:
                rp_s, rmap, _ = sr
                self._spmm(rp_s, self.send_st.col, sg1, gz, beta=1.0, row_map=rmap,
                           gate=h1[r0:r1])
            if self.agg0 is not None:
                a0 = self.agg0[r0:r1]
            else:
                a0 = self._agg(x, r0, r1, self.bufA[:n, :self.d0], "all", x_halo)
            s0, s1 = self.ch_S[ci]
            if v is None and s1 > s0:  # no room for v_self: scattered self term
                self._gemm(dZ[s0:s1], ws1_t, cin=gz, o_rows=self.ch_Sloc[ci],
                           gate=h1[r0:r1], out=gz)
            self.acc_in.add(x[r0:r1], gz, A2=a0)
        if not waited:
            self._mark("exchange_bwd_l0")
            work.wait()
            self._mark("bwd_l0")
        db0 = self.acc_in.col_result()
        self.edges_aggregated += self.nnz_it + \
            (self.nnz_h if (uh is not None or full) else
             self.send_st.nnz if self.send_st is not None else 0) + \
            (0 if self.agg0 is not None else self.nnz_it + self.nnz_h)
        w0 = self.acc_in.result()
        gw[(0, 0)], gw[(0, 1)], gw[(0, 2)] = (w0[:self.d0_in],
                                              w0[self.d0:self.d0 + self.d0_in], db0)
