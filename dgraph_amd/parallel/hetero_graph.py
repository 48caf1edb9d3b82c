"""Relation-stacked distributed aggregation for heterogeneous graphs (R-GCN hot path).

One :class:`SourceGraph` per SOURCE node type holds every relation that reads that type,
stacked by destination rows (``dgraph_amd.data.mag.build_hetero_partition``), over one
column space ``[local source rows | halo rows]``. So a layer moves each source type's halo
ONCE for all of its relations (the reference exchanged per relation and per gather/scatter
call, RGAT.py:171-201 — five collectives per relation-layer), and:

* ``static`` inputs (layer-0 vertex features: no gradient) fetch their halo rows once and
  keep them — through the symmetric heap's one-sided remote get when the features live on
  the heap (backend ``rocshmem``/``nvshmem``, K15 replacement), else one all-to-all-v;
* dynamic inputs (hidden activations) are packed with the native row gather and exchanged
  by RCCL all-to-all-v on the comm stream while the interior SpMMs of every relation run;
  only the halo SpMMs wait (the SAGE path's overlap, ``parallel/dist_graph.py``);
* backward is the exact adjoint: per-relation transposed SpMMs, halo rows accumulated into
  one ``[H, F]`` buffer and returned to their owners with ONE reverse all-to-all-v, then
  segment-summed (no float atomics).

Each relation reads its own column slice of the input, so the layer-0 transform-first path
(``Z = X_s [W_r1 | W_r2 ...]``, one GEMM per source type) and the aggregate-first path
(every relation reads all columns of ``h_s``) are the same Function.
"""
from __future__ import annotations

import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import torch
from torch.autograd import Function

from ..comm.alltoallv import AllToAllV
from ..ops import kernels as K
from ..ops.csr import CSR, IndexMap, _rowptr_from_sorted_rows, index_dtype_for


def _slice_rows(csr: CSR, lo: int, hi: int) -> CSR:
    """Rows [lo, hi) as a CSR whose column array is a view of ``csr.col``."""
    rp = csr.rowptr[lo:hi + 1]
    a, b = int(rp[0]), int(rp[-1])
    return CSR((rp - a).contiguous(), csr.col[a:b], csr.num_cols)


def _transpose_noperm(csr: CSR) -> CSR:
    """A^T without the slot permutation (unweighted aggregation only needs the pattern)."""
    cols = csr.col.long()
    ct, perm = torch.sort(cols, stable=True)
    rows = csr.row_ids()[perm].to(index_dtype_for(max(csr.num_rows, 1)))
    del perm
    return CSR(_rowptr_from_sorted_rows(ct, csr.num_cols), rows.contiguous(), csr.num_rows)


class SourceGraph:
    """All relations with one source node type, seen from one rank."""

    def __init__(self, csr: CSR, ranges: Dict[int, Tuple[int, int]], num_src_local: int,
                 num_halo: int, send_local_idx: Optional[torch.Tensor] = None,
                 send_splits: Optional[Sequence[int]] = None,
                 recv_splits: Optional[Sequence[int]] = None, group=None,
                 overlap: bool = True, halo_gids: Optional[torch.Tensor] = None,
                 src_offsets: Optional[Sequence[int]] = None):
        assert csr.num_cols == num_src_local + num_halo
        self.Ls, self.H = int(num_src_local), int(num_halo)
        self.ranges = {int(k): (int(v[0]), int(v[1])) for k, v in ranges.items()}
        self.inv_deg = csr.inv_degree()
        self.overlap = overlap
        self.halo_gids, self.src_offsets = halo_gids, src_offsets
        has_peers = self.H > 0 or (send_local_idx is not None and send_local_idx.numel() > 0)
        if has_peers:
            self.interior, self.halo = csr.split_columns(self.Ls)
            self.send_map = IndexMap(send_local_idx.to(csr.device), self.Ls)
            self.a2a = AllToAllV(send_splits, recv_splits, group)
            self.a2a_rev = self.a2a.reversed()
            if self.a2a.total_recv != self.H:
                raise ValueError(f"recv splits sum {self.a2a.total_recv} != halo {self.H}")
        else:
            self.interior, self.halo = csr, None
            self.send_map = self.a2a = self.a2a_rev = None
        self._slices: Dict[tuple, CSR] = {}
        self._static: dict = {}
        self.heap = None  # SymmetricHeap for one-sided static-halo fetches

    @staticmethod
    def from_partition(d: dict, group=None, overlap: bool = True,
                       src_offsets=None) -> "SourceGraph":
        return SourceGraph(d["csr"], d["ranges"], d["L"], d["H"], d["send_local_idx"],
                           d["send_splits"], d["recv_splits"], group, overlap,
                           d.get("halo_gids"), src_offsets)

    @property
    def device(self):
        return self.interior.device

    # ------------------------------------------------------------------ cached pieces
    def part(self, which: str, rid: int, transposed: bool = False) -> CSR:
        key = (which, rid, transposed)
        c = self._slices.get(key)
        if c is None:
            base = self.interior if which == "interior" else self.halo
            lo, hi = self.ranges[rid]
            c = _slice_rows(base, lo, hi)
            if transposed:
                c = _transpose_noperm(c)
            self._slices[key] = c
        return c

    def scale(self, rid: int) -> torch.Tensor:
        key = ("scale", rid)
        s = self._slices.get(key)
        if s is None:
            lo, hi = self.ranges[rid]
            s = self.inv_deg[lo:hi].contiguous()
            self._slices[key] = s
        return s

    def prepare_backward(self, rids: Optional[Sequence[int]] = None):
        for rid in (rids if rids is not None else self.ranges):
            self.part("interior", rid, True)
            if self.halo is not None:
                self.part("halo", rid, True)
        if self.send_map is not None:
            self.send_map.transpose_csr()
        return self

    # ------------------------------------------------------------------ halo rows
    def static_halo(self, x: torch.Tensor) -> Optional[torch.Tensor]:
        """Halo rows of a read-only input, fetched once and kept (keyed by a weak
        reference and the version counter, so in-place updates re-fetch). One-sided
        remote get from the owners' heaps when ``x`` lives on the attached heap."""
        if self.halo is None:
            return None
        c = self._static
        if c.get("ref") is not None and c["ref"]() is x and c["version"] == x._version:
            return c["recv"]
        c.clear()
        h = self.heap
        if h is not None and h.owns(x) and self.halo_gids is not None and x.is_cuda:
            recv = self._heap_get(h, x)
        else:
            recv = self.a2a(K.gather_rows(x, self.send_map.idx))
        c.update(ref=weakref.ref(x), version=x._version, recv=recv)
        return recv

    def _heap_get(self, heap, x: torch.Tensor) -> torch.Tensor:
        from .. import _native

        off = torch.as_tensor(self.src_offsets, dtype=torch.long, device=x.device)
        gids = self.halo_gids.to(x.device).long()
        owners = torch.bucketize(gids, off, right=True) - 1
        local = gids - off[owners]
        F = x.shape[1]
        out = torch.empty(gids.numel(), F, dtype=x.dtype, device=x.device)
        heap.barrier_stream()  # every owner's writes of x are visible (device-side)
        if out.numel():
            _native.ops().heap_get_rows(heap.table, heap.offset_of(x), owners, local, out,
                                        x.stride(0))
        heap.barrier_stream()  # no owner overwrites x while peers still read it
        return out

    # ------------------------------------------------------------------ forward / adjoint
    def forward_rels(self, z: torch.Tensor, z_halo: Optional[torch.Tensor],
                     spec: Sequence[Tuple[int, int, int]], mean: bool = True,
                     exchange: bool = True,
                     into: Optional[Sequence[torch.Tensor]] = None) -> List[torch.Tensor]:
        """``out_r = A_r[:, local] z[:, c0:c1] + A_r[:, halo] halo(z)[:, c0:c1]`` for every
        ``(r, c0, c1)`` in ``spec``. With ``exchange`` the halo rows of ``z`` are moved by
        an all-to-all-v overlapped with the interior SpMMs; else ``z_halo`` is used.
        ``into``: one existing tensor per spec entry that ``out_r`` is ADDED to (the
        destination's skip term: no separate output and add pass)."""
        recv, work = z_halo, None
        if self.halo is not None and exchange:
            recv, work = self.a2a(K.gather_rows(z, self.send_map.idx), async_op=True)
            if not self.overlap:
                work.wait()
        outs = []
        for i, (rid, c0, c1) in enumerate(spec):
            p = self.part("interior", rid)
            if into is not None:
                outs.append(K.spmm(p.rowptr, p.col, z[:, c0:c1], into[i],
                                   row_scale=self.scale(rid) if mean else None, beta=1.0))
                continue
            outs.append(K.spmm(p.rowptr, p.col, z[:, c0:c1],
                               row_scale=self.scale(rid) if mean else None))
        if self.halo is not None:
            if work is not None:
                work.wait()
            for (rid, c0, c1), o in zip(spec, outs):
                p = self.part("halo", rid)
                K.spmm(p.rowptr, p.col, recv[:, c0:c1], o,
                       row_scale=self.scale(rid) if mean else None, beta=1.0)
        return outs

    def backward_rels(self, grads: Sequence[Optional[torch.Tensor]],
                      spec: Sequence[Tuple[int, int, int]], width: int, dtype, mean: bool = True,
                      exchange: bool = True):
        """Adjoint of :meth:`forward_rels`: returns ``(gz [Ls, width], gz_halo or None)``."""
        dev = self.device

        def accumulate(which: str, nrows: int) -> torch.Tensor:
            buf = torch.empty(nrows, width, dtype=dtype, device=dev)
            written = torch.zeros(width, dtype=torch.bool)
            for (rid, c0, c1), g in zip(spec, grads):
                if g is None:
                    continue
                p = self.part(which, rid, transposed=True)
                first = not bool(written[c0:c1].any())
                if not first and not bool(written[c0:c1].all()):
                    raise ValueError("overlapping relation column slices must coincide")
                K.spmm(p.rowptr, p.col, g.contiguous(), buf[:, c0:c1],
                       col_scale=self.scale(rid) if mean else None, beta=0.0 if first else 1.0)
                written[c0:c1] = True
            if not bool(written.all()):
                for c in range(width):  # zero the untouched column runs
                    if not written[c]:
                        e = c
                        while e < width and not written[e]:
                            e += 1
                        buf[:, c:e].zero_()
                        written[c:e] = True
            return buf

        gz_halo = accumulate("halo", self.H) if self.halo is not None else None
        sg = work = None
        if gz_halo is not None and exchange:
            sg, work = self.a2a_rev(gz_halo, async_op=True)
            if not self.overlap:
                work.wait()
        gz = accumulate("interior", self.Ls)
        if sg is not None:
            work.wait()
            st = self.send_map.transpose_csr()
            K.spmm(st.rowptr, st.col, sg, gz, beta=1.0)
            gz_halo = None
        return gz, gz_halo


class _SourceAggFn(Function):
    @staticmethod
    def forward(ctx, z, z_halo, graph: SourceGraph, spec, mean: bool, exchange: bool):
        ctx.graph, ctx.spec, ctx.mean, ctx.exchange = graph, spec, mean, exchange
        ctx.width, ctx.dtype = z.shape[1], z.dtype
        ctx.has_halo = z_halo is not None
        outs = graph.forward_rels(z, z_halo, spec, mean, exchange)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        gz, gz_halo = ctx.graph.backward_rels(grads, ctx.spec, ctx.width, ctx.dtype, ctx.mean,
                                              ctx.exchange)
        return gz, (gz_halo if ctx.has_halo else None), None, None, None, None


class _SourceAggIntoFn(Function):
    @staticmethod
    def forward(ctx, z, z_halo, graph: SourceGraph, spec, mean: bool, exchange: bool,
                slots, *targets):
        ctx.graph, ctx.spec, ctx.mean, ctx.exchange = graph, spec, mean, exchange
        ctx.width, ctx.dtype = z.shape[1], z.dtype
        ctx.has_halo = z_halo is not None
        ctx.slots = slots
        graph.forward_rels(z, z_halo, spec, mean, exchange, into=[targets[i] for i in slots])
        ctx.mark_dirty(*targets)
        return targets

    @staticmethod
    def backward(ctx, *gts):
        grads = [gts[i] for i in ctx.slots]
        gz, gz_halo = ctx.graph.backward_rels(grads, ctx.spec, ctx.width, ctx.dtype, ctx.mean,
                                              ctx.exchange)
        return (gz, (gz_halo if ctx.has_halo else None), None, None, None, None, None, *gts)


def source_aggregate_into(z: torch.Tensor, graph: SourceGraph,
                          spec: Sequence[Tuple[int, int, int]],
                          targets: Sequence[torch.Tensor], mean: bool = True,
                          static_halo: Optional[torch.Tensor] = None) -> List[torch.Tensor]:
    """:func:`source_aggregate` whose per-relation results are ADDED in place to
    ``targets`` (one per spec entry; the same tensor may appear more than once). Returns
    the updated targets in spec order (autograd: the targets' gradients pass through)."""
    uniq: List[torch.Tensor] = []
    slots = []
    for t in targets:
        for j, u in enumerate(uniq):
            if u is t:
                slots.append(j)
                break
        else:
            slots.append(len(uniq))
            uniq.append(t)
    exchange = static_halo is None
    outs = _SourceAggIntoFn.apply(z.contiguous() if z.stride(1) != 1 else z, static_halo,
                                  graph, tuple(spec), mean, exchange, tuple(slots), *uniq)
    return [outs[j] for j in slots]


def source_aggregate(z: torch.Tensor, graph: SourceGraph,
                     spec: Sequence[Tuple[int, int, int]], mean: bool = True,
                     static_halo: Optional[torch.Tensor] = None) -> List[torch.Tensor]:
    """Autograd entry: per-relation mean (or sum) aggregation of column slices of ``z``.
    ``static_halo`` (the halo rows of ``z``, already fetched) switches off the exchange;
    its gradient is returned to whoever produced it (no communication)."""
    exchange = static_halo is None
    outs = _SourceAggFn.apply(z.contiguous() if z.stride(1) != 1 else z, static_halo, graph,
                              tuple(spec), mean, exchange)
    return list(outs)
