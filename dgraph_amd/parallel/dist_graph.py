"""Per-rank partitioned graph with halo-overlapped aggregation.

This is the hot path of vertex-partitioned full-graph training (P1-P3, §5.7 design 1).
The local CSR (rows = owned vertices, columns = owned vertices ++ halo rows) is split
once into an *interior* part (columns < L) and a *halo* part (columns >= L). Then

    aggregate(x):   pack send rows (native gather) -> RCCL all-to-all-v on the comm stream
                    || interior SpMM on the compute stream -> wait -> halo SpMM (beta=1)
    aggregate_T(g): halo^T SpMM -> reverse all-to-all-v || interior^T SpMM -> wait ->
                    segment-sum of the received rows into their owners (beta=1)

so the interior aggregation hides the exchange, and there is no host sync and no float
atomic anywhere. ``aggregate_T`` is the exact adjoint of ``aggregate``. The reference
serialised every exchange with compute and synced the host per exchange (§3.2 notes).
"""
from __future__ import annotations

import os
import weakref
from dataclasses import dataclass
from typing import List, Optional

import torch
from torch.autograd import Function

from ..comm.alltoallv import AllToAllV
from ..ops import kernels as K
from ..ops.csr import CSR, IndexMap


# Hub-row split threshold for the SpMM (ops.csr.CSR.hub_split): rows with more entries
# run their tails as separate segment waves. 0 disables.
SPMM_HUB_CAP = int(os.environ.get("DGRAPH_SPMM_HUB_CAP", "2048"))


def _hs(csr: CSR):
    return csr.hub_split(SPMM_HUB_CAP) if SPMM_HUB_CAP > 0 else None


def _select_columns(csr: CSR, cols: torch.Tensor, ncols: int) -> CSR:
    """``csr`` restricted to the entries whose column is in ``cols`` (row order and the
    order within a row kept). Two passes over row chunks of ~2^26 entries: count, then
    copy into the exact-size column array (bounded temporaries at 10^9+ entries, no
    concatenation copy)."""
    dev = csr.device
    keep = torch.zeros(ncols, dtype=torch.bool, device=dev)
    keep[cols] = True
    R = csr.num_rows
    nnz = max(csr.col.numel(), 1)
    step = max(1, int(R * (1 << 26) // nnz))
    chunks = [(r0, min(R, r0 + step)) for r0 in range(0, R, step)]
    deg = torch.zeros(R, dtype=torch.long, device=dev)
    for r0, r1 in chunks:
        a, b = int(csr.rowptr[r0]), int(csr.rowptr[r1])
        if b == a:
            continue
        m = keep[csr.col[a:b].long()]
        rows = torch.repeat_interleave(torch.arange(r0, r1, device=dev),
                                       csr.rowptr[r0 + 1:r1 + 1] - csr.rowptr[r0:r1],
                                       output_size=b - a)
        deg[r0:r1] = torch.bincount(rows[m] - r0, minlength=r1 - r0)
        del m, rows
    rowptr = torch.zeros(R + 1, dtype=torch.long, device=dev)
    torch.cumsum(deg, 0, out=rowptr[1:])
    del deg
    col = torch.empty(int(rowptr[-1]), dtype=csr.col.dtype, device=dev)
    for r0, r1 in chunks:
        a, b = int(csr.rowptr[r0]), int(csr.rowptr[r1])
        if b == a:
            continue
        c = csr.col[a:b]
        col[int(rowptr[r0]):int(rowptr[r1])] = c[keep[c.long()]]
        del c
    return CSR(rowptr, col, csr.num_cols, None, symmetric=False)


def _cache_lookup(cache: dict, rows: torch.Tensor):
    """Plan-cache hit for the row-index tensor ``rows``: the SAME live tensor object (a
    weak reference, never the address, which a freed tensor's successor can reuse) at the
    same version counter (an in-place edit of ``rows`` misses). Building a sub-plan on a
    miss is collective, so the key must not depend on allocator state that can differ
    between ranks."""
    ref = cache.get("ref")
    if ref is not None and ref() is rows and cache.get("version") == rows._version:
        return cache["plan"]
    return None


def _cache_store(cache: dict, rows: torch.Tensor, plan) -> None:
    cache.clear()
    cache.update(ref=weakref.ref(rows), version=rows._version, plan=plan)


class DistGraph:
    def __init__(
        self,
        csr: CSR,
        num_local: int,
        num_halo: int,
        send_local_idx: Optional[torch.Tensor] = None,
        send_splits: Optional[List[int]] = None,
        recv_splits: Optional[List[int]] = None,
        group=None,
        symmetric: bool = False,
        overlap: bool = True,
        chunk_bytes: Optional[int] = None,
    ):
        assert csr.num_rows == num_local, "CSR rows must be the local vertices"
        assert csr.num_cols == num_local + num_halo
        self.L, self.H = int(num_local), int(num_halo)
        self.csr = csr
        self.inv_deg = csr.inv_degree()
        self.symmetric = symmetric
        self.overlap = overlap
        # per-peer message size above which an exchange is cut into column chunks
        self.chunk_bytes = int(os.environ.get("DGRAPH_HALO_CHUNK_BYTES", str(32 << 20))) \
            if chunk_bytes is None else int(chunk_bytes)
        self._restrict_cache = {}
        self._restrict_fwd_cache = {}
        self._static_cache = {}
        self._support_cache = {}
        # edges (nonzeros) aggregated by every call so far, forward and transposed:
        # bench.py reports the per-step delta as ``edges_aggregated_per_step``
        self.edges_aggregated = 0
        if self.H > 0 or (send_local_idx is not None and send_local_idx.numel() > 0):
            self.interior, self.halo = csr.split_columns(self.L)
            self.interior.symmetric = symmetric
            self.send_map = IndexMap(send_local_idx.to(csr.device), self.L)
            self.a2a = AllToAllV(send_splits, recv_splits, group)
            self.a2a_rev = self.a2a.reversed()
            if self.a2a.total_recv != self.H:
                raise ValueError(f"recv splits sum {self.a2a.total_recv} != halo {self.H}")
        else:
            self.interior, self.halo = csr, None
            self.interior.symmetric = symmetric
            self.send_map = None
            self.a2a = self.a2a_rev = None
        # drop the un-split copy's column array when split (memory: 288 GB budget)
        if self.halo is not None:
            self.csr = None
        from ..utils.diagnostics import maybe_validate

        maybe_validate(self)  # DGRAPH_CHECK_PLANS=1: once per plan, not per call

    @property
    def device(self):
        return self.interior.device if self.interior is not None else self._device

    @property
    def nnz(self) -> int:
        """Message edges aggregated at this rank's vertices (interior + halo)."""
        if self.interior is None:
            return self._nnz
        return self.interior.nnz + (self.halo.nnz if self.halo is not None else 0)

    def release_csr(self) -> None:
        """Drop the interior / halo CSRs (and everything cached from them). For an executor
        that built its own adjacency from them (models/sage_fused.py keeps a rank's interior
        and halo entries in ONE array) and needs only the exchange plans from here on: at
        the papers100M shape the split copy is 6.5 GB per rank at W = 2. The aggregation
        methods of this object cannot be used afterwards."""
        if self.interior is None:
            return
        self._device = self.interior.device
        self._nnz = self.nnz
        self._had_halo = self.halo is not None
        self.interior = None
        self.halo = None
        self._restrict_cache.clear()
        self._restrict_fwd_cache.clear()
        self._support_cache.clear()

    @staticmethod
    def from_pattern(cp, num_nbr_rows: Optional[int] = None, group=None,
                     symmetric: bool = False) -> "DistGraph":
        """From a :class:`CommunicationPattern` (its local_edge_list = (central, nbr))."""
        le = cp.local_edge_list
        L_n = cp.num_local_neighbor_vertices or cp.num_local_vertices
        if L_n != cp.num_local_vertices:
            raise ValueError("DistGraph needs a homogeneous pattern (use plan ops for bipartite)")
        csr = CSR.from_coo(le[:, 0], le[:, 1], cp.num_local_vertices,
                           cp.num_local_vertices + cp.num_halo_vertices)
        return DistGraph(csr, cp.num_local_vertices, cp.num_halo_vertices, cp.send_local_idx,
                         cp.send_splits(), cp.recv_splits(), group, symmetric)

    # ------------------------------------------------------------------ non-autograd
    def _static_halo(self, x: torch.Tensor) -> Optional[torch.Tensor]:
        """Halo rows of a read-only input (the vertex features), replicated once and kept:
        partition-time halo replication of inputs, as DistDGL-style partitions store them.
        Keyed by storage, shape and the tensor's version counter, so an in-place update of
        ``x`` re-exchanges."""
        c = self._static_cache
        if c.get("ref") is not None and c["ref"]() is x and c["version"] == x._version:
            return c["recv"]
        # a weak reference, not the address: a freed tensor's storage can be reused
        c.clear()
        cb = self.static_halo_block(x.shape[1], x.element_size())
        if cb >= x.shape[1]:
            recv = self.a2a(K.gather_rows(x, self.send_map.idx))
        else:
            # a large halo (structureless graph): packed and exchanged in column blocks, so
            # the transient send/receive buffers stay small next to the kept halo rows
            recv = torch.empty(self.a2a.total_recv, x.shape[1], dtype=x.dtype, device=x.device)
            for c0 in range(0, x.shape[1], cb):
                c1 = min(c0 + cb, x.shape[1])
                recv[:, c0:c1] = self.a2a(K.gather_rows(x[:, c0:c1], self.send_map.idx))
        c.update(ref=weakref.ref(x), version=x._version, recv=recv)
        return c["recv"]

    STATIC_BLOCK_BYTES = 4 << 30

    def static_halo_block(self, F: int, elem: int = 4) -> int:
        """Column-block width of the static halo exchange: whole rows unless the packed send
        rows exceed ``STATIC_BLOCK_BYTES``. Its transient (send + receive blocks) is
        ``(n_send + H) * block * elem`` bytes on top of the kept ``H * F`` halo rows."""
        n_send = self.send_map.idx.numel() if self.send_map is not None else 0
        if n_send * F * elem <= self.STATIC_BLOCK_BYTES:
            return F
        cb = max(16, (self.STATIC_BLOCK_BYTES // max(n_send * elem, 1)) // 16 * 16)
        return min(cb, F)

    def aggregate(self, x: torch.Tensor, mean: bool = True,
                  out: Optional[torch.Tensor] = None, static: bool = False,
                  halo_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Mean (or sum) over in-neighbours, local and halo. ``static=True`` marks ``x``
        as a read-only input whose halo rows may be exchanged once and reused.
        ``halo_rows``: the halo rows' values ``[H, F]`` computed on this rank (halo
        recomputation, :mod:`~dgraph_amd.parallel.halo_recompute`): no exchange."""
        rs = self.inv_deg if mean else None
        self.edges_aggregated += self.nnz
        if self.halo is None:
            return K.spmm(self.interior.rowptr, self.interior.col, x, out, row_scale=rs,
                          split=_hs(self.interior))
        if static or halo_rows is not None:
            recv = self._static_halo(x) if halo_rows is None else halo_rows
            out = K.spmm(self.interior.rowptr, self.interior.col, x, out, row_scale=rs,
                         split=_hs(self.interior))
            hc = self.halo.compact_rows()
            K.spmm(hc.rowptr, hc.col, recv, out, row_scale=rs, beta=1.0, split=_hs(hc),
                   row_map=hc.row_map)
            return out
        if out is None:
            out = torch.empty(self.L, x.shape[1], dtype=x.dtype, device=x.device)
        # column chunks: chunk k's halo SpMM runs while chunk k+1 is on the links
        pend = []
        for c0, c1 in self._col_chunks(self.a2a, x.shape[1], x.element_size()):
            xc = x if (c0, c1) == (0, x.shape[1]) else x[:, c0:c1]
            recv, work = self.a2a(K.gather_rows(xc, self.send_map.idx), async_op=True)
            if not self.overlap:
                work.wait()
            pend.append((c0, c1, recv, work))
        K.spmm(self.interior.rowptr, self.interior.col, x, out, row_scale=rs,
               split=_hs(self.interior))
        hc = self.halo.compact_rows()
        for c0, c1, recv, work in pend:
            work.wait()
            oc = out if (c0, c1) == (0, x.shape[1]) else out[:, c0:c1]
            K.spmm(hc.rowptr, hc.col, recv, oc, row_scale=rs, beta=1.0, split=_hs(hc),
                   row_map=hc.row_map)
        return out

    def _col_chunks(self, a2a, F: int, esize: int):
        """Column ranges of one exchange: a single range unless the largest per-peer
        message exceeds 2 x ``chunk_bytes``; then chunks of whole 64-column blocks, each
        per-peer message of a chunk >= ``chunk_bytes`` / 2 (RCCL's per-call cost stays
        negligible; xGMI is point-to-point, so a peer message is one link's load)."""
        cb = self.chunk_bytes
        peer = max(max(a2a.send_splits, default=0), max(a2a.recv_splits, default=0))
        per_peer = peer * F * esize
        if cb <= 0 or per_peer <= 2 * cb or F < 128:
            return [(0, F)]
        n = min(-(-per_peer // cb), F // 64)
        w = -(-F // n)
        w = -(-w // 64) * 64
        return [(c, min(c + w, F)) for c in range(0, F, w)]

    # row blocks of the fused pre-scale + bias-gradient column sums (row_scale_colsum)
    COLSUM_BLOCKS = 1024

    @staticmethod
    def _spmm_col_scaled(csr: CSR, g: torch.Tensor, cs: torch.Tensor, out, scratch,
                         colsum: Optional[list] = None):
        """``A g`` with a column scale. With a ``scratch`` buffer (a free workspace slot)
        the scale is applied to column slices of ``g`` first (one streaming pass) and the
        SpMM runs unweighted: a per-edge scale gather costs the gather-bound kernel a
        second scattered load per neighbour (+25-55 % per pass, benchmarks/bench_spmm.py
        --mean col)."""
        rows, F = g.shape
        S = 0 if scratch is None else min(F, (scratch.numel() // max(rows, 1)) // 64 * 64)
        if S < 64 or g.dtype != torch.bfloat16 or not g.is_cuda:
            out = K.spmm(csr.rowptr, csr.col, g, out, col_scale=cs, split=_hs(csr))
            if colsum is not None:
                colsum.append(K.col_sum(g))
            return out
        if out is None:
            out = torch.empty(csr.num_rows, F, dtype=g.dtype, device=g.device)
        aligned = g.data_ptr() % 16 == 0 and scratch.data_ptr() % 16 == 0 and F % 8 == 0
        # ``colsum`` (a list): append the fp32 column sums of g, formed by the scale pass
        partial = None
        if colsum is not None and aligned and F <= 2048:
            partial = torch.empty(min(DistGraph.COLSUM_BLOCKS, max(rows, 1)), F,
                                  dtype=torch.float32, device=g.device)
        for c0 in range(0, F, S):
            w = min(S, F - c0)
            buf = scratch[: rows * w].view(rows, w)
            if partial is not None and w % 8 == 0 and w <= 256:
                K.row_scale_colsum(g[:, c0:c0 + w], cs, buf, partial[:, c0:c0 + w])
            elif aligned and w % 8 == 0:
                if partial is not None:
                    partial[:, c0:c0 + w].zero_()
                    partial[0, c0:c0 + w] = K.col_sum(g[:, c0:c0 + w])
                K.row_scale_cols(g[:, c0:c0 + w], cs, buf)
            else:
                torch.mul(g[:, c0:c0 + w], cs.unsqueeze(1), out=buf)
            K.spmm(csr.rowptr, csr.col, buf, out[:, c0:c0 + w], split=_hs(csr))
        if colsum is not None:
            colsum.append(partial.sum(0) if partial is not None else K.col_sum(g))
        return out

    def _interior_T(self, it: CSR, g, cs, out, scratch, colsum):
        if cs is not None and scratch is not None:
            return self._spmm_col_scaled(it, g, cs, out, scratch.reshape(-1), colsum)
        out = K.spmm(it.rowptr, it.col, g, out, col_scale=cs, split=_hs(it))
        if colsum is not None:
            colsum.append(K.col_sum(g))
        return out

    def aggregate_T(self, g: torch.Tensor, mean: bool = True,
                    out: Optional[torch.Tensor] = None,
                    scratch: Optional[torch.Tensor] = None, overlap=None,
                    halo_out: Optional[torch.Tensor] = None,
                    colsum: Optional[list] = None, support=None) -> torch.Tensor:
        """Transposed aggregation (the backward of :meth:`aggregate`). ``scratch``: an
        optional free buffer (any shape, same dtype as ``g``) for the pre-scaled path.
        ``overlap``: a callable of independent work, run after the reverse exchange and
        the interior SpMM are issued and before the exchange is waited for.
        ``halo_out``: ``[H, F]`` buffer that receives the halo rows' gradient, which then
        stays on this rank (halo recomputation: the rows were computed here) — no
        exchange, no owner-side segment sum. ``colsum``: a list that receives the fp32
        column sums of ``g`` (a bias gradient) before ``overlap`` runs — formed by the
        pre-scale pass when there is one, else by a column-sum pass."""
        cs = self.inv_deg if mean else None
        g = g.contiguous()
        it = self.interior if self.interior.symmetric else self.interior.transpose()
        if support is not None:
            # ``support`` = grad_support(rows): g is zero outside S, so only the interior
            # entries with a source in S contribute
            it = support[1]
        self.edges_aggregated += it.nnz + (self.halo.nnz if self.halo is not None else 0)
        if halo_out is not None and self.halo is not None:
            K.spmm(self.halo.transpose().rowptr, self.halo.transpose().col, g, halo_out,
                   col_scale=cs, split=_hs(self.halo.transpose()))
            out = self._interior_T(it, g, cs, out, scratch, colsum)
            if overlap is not None:
                overlap()
            return out
        if self.halo is None:
            out = self._interior_T(it, g, cs, out, scratch, colsum)
            if overlap is not None:
                overlap()
            return out
        ht = self.halo.transpose()
        F = g.shape[1]
        pend = []
        for c0, c1 in self._col_chunks(self.a2a_rev, F, g.element_size()):
            gc = g if (c0, c1) == (0, F) else g[:, c0:c1]
            hg = K.spmm(ht.rowptr, ht.col, gc, col_scale=cs, split=_hs(ht))
            sg, work = self.a2a_rev(hg, async_op=True)
            if not self.overlap:
                work.wait()
            pend.append((c0, c1, sg, work))
        out = self._interior_T(it, g, cs, out, scratch, colsum)
        if overlap is not None:
            overlap()  # independent work queued behind the exchange (e.g. a weight grad)
        st = self.send_map.transpose_csr().compact_rows()
        for c0, c1, sg, work in pend:
            work.wait()
            oc = out if (c0, c1) == (0, F) else out[:, c0:c1]
            K.spmm(st.rowptr, st.col, sg, oc, beta=1.0, split=_hs(st), row_map=st.row_map)
        return out

    def _peers(self) -> bool:
        """True when the plan's peers exist (a process group of the plan's size)."""
        import torch.distributed as dist

        return dist.is_initialized() and dist.get_world_size(self.a2a.group) > 1

    def _restricted(self, rows: torch.Tensor):
        """Cached pieces of :meth:`aggregate_T_rows` for one loss-row set: the transposed
        interior block A[rows, :L]^T, and for the halo block only the halo rows that
        neighbour a loss row (A[rows, halo]^T restricted to its nonzero rows) with a
        matching sub-plan of the reverse exchange, so the owners receive just those rows
        instead of all H (built once, collectively: two small all-to-alls)."""
        hit = _cache_lookup(self._restrict_cache, rows)
        if hit is not None:
            return hit
        it = self.interior.select_rows(rows).transpose()
        cs = self.inv_deg[rows.long()].contiguous()
        sub = None
        if self.halo is not None:
            from ..plan.pattern import _alltoall_counts, _alltoallv_ids

            ht = self.halo.select_rows(rows).transpose()  # [H, |rows|]
            nz = torch.nonzero(ht.degree() > 0).reshape(-1)
            ht_nz = ht.select_rows(nz)
            dev = nz.device
            recv_off = torch.zeros(len(self.a2a.recv_splits) + 1, dtype=torch.long, device=dev)
            recv_off[1:] = torch.cumsum(torch.tensor(self.a2a.recv_splits, device=dev), 0)
            owner = torch.searchsorted(recv_off[1:], nz, right=True)
            W = recv_off.numel() - 1
            cnt = torch.bincount(owner, minlength=W)
            slot = nz - recv_off[owner]
            if self._peers():
                peer_cnt = _alltoall_counts(cnt, self.a2a.group)
            else:  # single-process rehearsal of a W-way rank: mirrored loopback plan
                peer_cnt = cnt.clone()
            cnt_l, peer_l = [int(v) for v in cnt.tolist()], [int(v) for v in peer_cnt.tolist()]
            send_sp = torch.tensor(self.a2a.send_splits, device=dev)
            if self._peers():
                peer_slot = _alltoallv_ids(slot, cnt_l, peer_l, self.a2a.group)
            else:
                # mirrored loopback: peer p's request for slot s lands in my send segment for
                # p (whose length may differ from what I receive from p)
                peer_slot = slot % send_sp[owner].clamp_min(1)
            send_off = torch.zeros(W + 1, dtype=torch.long, device=dev)
            send_off[1:] = torch.cumsum(send_sp, 0)
            base = torch.repeat_interleave(send_off[:-1], peer_cnt.to(dev))
            recv_local = self.send_map.idx.long()[base + peer_slot.to(dev)]
            sub = (ht_nz, AllToAllV(cnt_l, peer_l, self.a2a.group),
                   IndexMap(recv_local, self.L).transpose_csr(), nz, recv_local)
        hit = (it, cs, sub)
        _cache_store(self._restrict_cache, rows, hit)  # one loss-row set at a time
        return hit

    def aggregate_T_rows(self, g_rows: torch.Tensor, rows: torch.Tensor, mean: bool = True,
                         out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``aggregate_T(g)`` for a ``g`` that is zero outside ``rows`` (given as the
        ``[len(rows), F]`` nonzero block): the transposed SpMM over A[rows, :] only. For an
        output layer trained on 1 % of the vertices this reads ~1 % of the edges and sends
        back only the halo rows that carry a contribution, with exactly the result of the
        dense call. The first call for a row set is collective (sub-plan exchange)."""
        it, cs_rows, sub = self._restricted(rows)
        g_rows = g_rows.contiguous()
        if mean:
            # the column scale applies to the |rows| gradient rows: scale them once (a
            # 1 %-of-V pass) instead of gathering a per-edge scale inside the SpMM
            g_rows = (g_rows.float() * cs_rows.unsqueeze(1)).to(g_rows.dtype) \
                if g_rows.dtype != torch.float64 else g_rows * cs_rows.unsqueeze(1)
        self.edges_aggregated += it.nnz + (sub[0].nnz if sub is not None else 0)
        # A[rows, :]^T touches only the ~30 % of vertices adjacent to a loss row: run the
        # SpMM over those rows (row-compacted, output row map) and zero-fill the rest,
        # instead of walking all V rows of a 1 %-dense transposed block
        itc = it.compact_rows()
        if out is None:
            out = torch.empty(it.num_rows, g_rows.shape[1], dtype=g_rows.dtype,
                              device=g_rows.device)
        out.zero_()
        if sub is None:
            K.spmm(itc.rowptr, itc.col, g_rows, out, split=_hs(itc), row_map=itc.row_map)
            return out
        ht_nz, a2a_sub, st = sub[:3]
        hg = K.spmm(ht_nz.rowptr, ht_nz.col, g_rows, split=_hs(ht_nz))
        sg, work = a2a_sub(hg, async_op=True)
        if not self.overlap:
            work.wait()
        K.spmm(itc.rowptr, itc.col, g_rows, out, split=_hs(itc), row_map=itc.row_map)
        work.wait()
        K.spmm(st.rowptr, st.col, sg, out, beta=1.0, split=_hs(st))
        return out

    # gradient-support restriction of the transposed aggregation (see grad_support); off
    # with DGRAPH_GRAD_SUPPORT=0. Built only with this much device memory left over.
    GRAD_SUPPORT = os.environ.get("DGRAPH_GRAD_SUPPORT", "1") != "0"
    SUPPORT_HEADROOM = 12 << 30

    def grad_support(self, rows: torch.Tensor):
        """The :meth:`prepare_grad_support` result for ``rows`` (``None`` when it was not
        prepared for this row tensor: then the full transposed block is used)."""
        return _cache_lookup(self._support_cache, rows)

    def prepare_grad_support(self, rows: torch.Tensor):
        """For a loss on ``rows`` with a project-first output layer: the local rows where
        the gradient entering the layer below the output layer can be nonzero — the loss
        rows and their in-neighbours (the rows :meth:`aggregate_T_rows` writes, plus the
        rows the halo sub-plan adds to), and the interior transposed block restricted to
        those columns, ``A^T[:, S]`` (cached per ``rows``, like the restricted plans).

        The transposed aggregation of that gradient then walks only the edges whose
        source lies in S (~30 % of them on the bench graph): exact, the other terms are
        products with rows that are zero by construction. Returns ``None`` when disabled
        or when the restricted block does not fit in device memory. Build it at setup,
        before the training workspace exists (bench.py does so on partitioned graphs; on
        one GPU at the papers100M shape the extra ~5 GB pushed the caching allocator into
        per-step release/re-map stalls: 791 -> 853 ms although the kernels got 80 ms
        faster). Collective on a partitioned graph (the restricted plan)."""
        if not self.GRAD_SUPPORT:
            return None
        hit = _cache_lookup(self._support_cache, rows)
        if hit is not None:
            return hit
        it, _, sub = self._restricted(rows)
        parts = [rows.long(), it.compact_rows().row_map.long()]
        if sub is not None:
            parts.append(sub[4].long())  # local rows the halo sub-plan adds to
        S = torch.unique(torch.cat(parts))
        full = self.interior if self.interior.symmetric else self.interior.transpose()
        res = None
        dev = full.device
        keep_frac = S.numel() / max(self.L, 1)
        # the kept columns (~|S|/L of the entries) + row pointers + chunk temporaries
        need = int(full.col.numel() * keep_frac * 1.1) * full.col.element_size() + \
            2 * full.rowptr.numel() * 8 + (1 << 30)
        free = torch.cuda.mem_get_info(dev)[0] if dev.type == "cuda" else need + (64 << 30)
        if free - need >= self.SUPPORT_HEADROOM:
            res = (S, _select_columns(full, S, self.L))
        _cache_store(self._support_cache, rows, res)
        return res

    def _restricted_fwd(self, rows: torch.Tensor):
        """Forward counterpart of :meth:`_restricted`: A[rows, :L] and A[rows, halo] with
        the halo columns renumbered onto the contributing halo rows only, plus the
        forward sub-plan (owners send just those rows: the reverse of the backward
        sub-plan)."""
        hit = _cache_lookup(self._restrict_fwd_cache, rows)
        if hit is not None:
            return hit
        ir = self.interior.select_rows(rows)
        rs = self.inv_deg[rows.long()].contiguous()
        hsub = None
        if self.halo is not None:
            _, _, sub = self._restricted(rows)
            _, a2a_sub, _, nz, recv_local = sub
            hr = self.halo.select_rows(rows)
            pos = torch.full((self.H,), -1, dtype=torch.long, device=nz.device)
            pos[nz] = torch.arange(nz.numel(), device=nz.device)
            hr = CSR(hr.rowptr, pos[hr.col.long()].to(torch.int32).contiguous(),
                     max(int(nz.numel()), 1))
            hsub = (hr, a2a_sub.reversed(), recv_local.to(self.send_map.idx.dtype))
        hit = (ir, rs, hsub)
        _cache_store(self._restrict_fwd_cache, rows, hit)
        return hit

    def aggregate_rows(self, x: torch.Tensor, rows: torch.Tensor, mean: bool = True,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``aggregate(x)[rows]`` without aggregating the other rows: A[rows, :] x over the
        interior block, and over only the halo rows that neighbour ``rows`` (the owners
        send just those, overlapped with the interior SpMM). The first call for a row set
        is collective (sub-plan exchange, shared with :meth:`aggregate_T_rows`)."""
        ir, rs, hsub = self._restricted_fwd(rows)
        rsc = rs if mean else None
        self.edges_aggregated += ir.nnz + (hsub[0].nnz if hsub is not None else 0)
        if hsub is None:
            return K.spmm(ir.rowptr, ir.col, x, out, row_scale=rsc, split=_hs(ir))
        hr, a2a_f, recv_local = hsub
        recv, work = a2a_f(K.gather_rows(x, recv_local), async_op=True)
        if not self.overlap:
            work.wait()
        out = K.spmm(ir.rowptr, ir.col, x, out, row_scale=rsc, split=_hs(ir))
        work.wait()
        K.spmm(hr.rowptr, hr.col, recv, out, row_scale=rsc, beta=1.0, split=_hs(hr))
        return out

    def prepare_backward(self):
        """Build the cached transposes and hub-row splits eagerly (outside any timed
        region)."""
        csrs = [self.interior]
        if not self.interior.symmetric:
            csrs.append(self.interior.transpose())
        if self.halo is not None:
            csrs += [self.halo.compact_rows(), self.halo.transpose(),
                     self.send_map.transpose_csr().compact_rows()]
        for c in csrs:
            _hs(c)
        return self

    def memory_bytes(self) -> int:
        n = self.interior.memory_bytes()
        if self.halo is not None:
            n += self.halo.memory_bytes()
        return n


class _DistAggregateFn(Function):
    @staticmethod
    def forward(ctx, x, graph: DistGraph, mean: bool):
        ctx.graph, ctx.mean = graph, mean
        return graph.aggregate(x.contiguous(), mean)

    @staticmethod
    def backward(ctx, g):
        return ctx.graph.aggregate_T(g, ctx.mean), None, None


def dist_aggregate(x: torch.Tensor, graph: DistGraph, mean: bool = True) -> torch.Tensor:
    """Autograd-aware distributed neighbourhood aggregation (sum or mean)."""
    return _DistAggregateFn.apply(x, graph, mean)
