"""Halo recomputation: trade first-layer compute for xGMI link bytes.

A W-way vertex partition exchanges, per training step of an L-layer GraphSAGE, the halo
rows of every hidden layer forward and their gradients backward (the input features'
halo is static and moves once). On the papers100M-shaped graph at W=2 that is
256 + 192 + 256 columns x 23.3 M halo rows = 32.8 GB over ONE point-to-point xGMI link per
step (PERFORMANCE.md): more link time than the rank's whole compute.

With halo recomputation a rank computes the first hidden layer ``h1`` for its halo
vertices itself, from their full neighbourhoods (static input features of the 1- and
2-hop halo, fetched once). Layer 2 then reads ``h1[halo]`` locally, and the gradient that
flows into ``h1[halo]`` stays local too: it feeds this rank's own first-layer weight
gradient, and the weight all-reduce sums every rank's share exactly as before (the
owner back-propagates only its own uses of the row). Result: the layer-2 forward
exchange and the layer-2 backward exchange disappear; only the output layer's halo moves
(192 of 704 columns at the bench shape). Cost: the first layer runs on L + H rows, and
the halo rows' neighbourhood lists and 2-hop features are held once.

Exact (not an approximation): same arithmetic per row; bench.py ``--halo-recompute``
decides per shape (on when the halo is smaller than the partition: W = 2, 4 on the bench
graph). Row layout of the extended first layer (``Lp`` = L rounded up to 256, so the
1-bit ReLU masks of the two row ranges fall in separate 256-row mask groups of the MFMA
epilogue's tile32 layout)::

    [0, L) owned rows | [L, Lp) zero padding | [Lp, Lp + H) halo rows | (inputs only:)
    [Lp + H, Lp + H + H2) 2-hop halo rows

Reference: no equivalent (the reference always exchanges every layer,
``DGraph/distributed/nccl/NCCLBackendEngine.py:281-306``).
"""
from __future__ import annotations

import os
import weakref
from typing import List, Optional

import torch

from ..comm.alltoallv import AllToAllV
from ..ops import kernels as K
from ..ops.csr import CSR
from .dist_graph import DistGraph, _hs

# owned rows aggregated in one pass over the merged (interior + halo) CSR; 0 = the
# interior pass + a beta=1 halo pass (DGRAPH_RECOMPUTE_MERGED)
MERGED = os.environ.get("DGRAPH_RECOMPUTE_MERGED", "1") != "0"


class HaloRecompute:
    """First-layer rows and inputs of halo recomputation for one rank of ``graph``.

    ``rows_csr``: CSR over this rank's halo vertices (``halo_gids``, sorted, the order of
    ``graph``'s halo columns) with GLOBAL column ids — each halo vertex's full
    neighbourhood. ``offsets``: contiguous ownership ranges. Collective over ``group``
    (the 2-hop fetch plan) unless ``rehearse`` (one rank alone: loopback plan of the
    right size, as bench.py --rehearse-world)."""

    def __init__(self, graph: DistGraph, rows_csr: CSR, halo_gids: torch.Tensor,
                 offsets: List[int], rank: int, group=None, rehearse: bool = False):
        from ..plan.pattern import _alltoall_counts, _alltoallv_ids

        if graph.halo is None:
            raise ValueError("halo recomputation needs a partitioned graph")
        L, H = graph.L, graph.H
        if rows_csr.num_rows != H or halo_gids.numel() != H:
            raise ValueError("rows_csr must have one row per halo vertex")
        self.graph = graph
        self.L, self.H = L, H
        self.Lp = (L + 255) // 256 * 256  # tile32 masks come in 256-row groups
        self.L1 = self.Lp + H
        dev = rows_csr.device
        lo, hi = offsets[rank], offsets[rank + 1]
        hg = halo_gids.to(dev).long()
        c = rows_csr.col.long()
        local = (c >= lo) & (c < hi)
        pos = torch.searchsorted(hg, c).clamp_(max=max(H - 1, 0))
        in_halo = (~local) & (hg[pos] == c)
        other = ~(local | in_halo)
        halo2 = torch.unique(c[other])
        del other
        self.H2 = int(halo2.numel())
        p2 = torch.searchsorted(halo2, c) if self.H2 else torch.zeros_like(c)
        newc = torch.where(local, c - lo, torch.where(in_halo, self.Lp + pos, self.L1 + p2))
        del c, pos, p2, local, in_halo
        ncols = self.L1 + self.H2
        idt = torch.int32 if ncols < 2**31 else torch.int64
        self.csr = CSR(rows_csr.rowptr, newc.to(idt), ncols, None, symmetric=False)
        del newc
        self.inv_deg = self.csr.inv_degree()
        # 2-hop input rows: fetched once from their owners
        W = len(offsets) - 1
        off_t = torch.tensor(offsets, device=dev, dtype=torch.int64)
        owners = torch.bucketize(halo2, off_t, right=True) - 1
        recv_splits = torch.bincount(owners, minlength=W).tolist() if self.H2 else [0] * W
        if rehearse:
            send_splits = list(recv_splits)
            n = sum(send_splits)
            send_idx = torch.arange(n, device=dev, dtype=torch.long) * 7919 % max(L, 1)
        else:
            req = torch.tensor(recv_splits, dtype=torch.long, device=dev)
            send_splits = [int(v) for v in _alltoall_counts(req, group).tolist()]
            send_idx = _alltoallv_ids(halo2, recv_splits, send_splits, group) - lo
        self.send_idx2 = send_idx.to(torch.int32 if L < 2**31 else torch.int64)
        self.a2a2 = AllToAllV(send_splits, recv_splits, group)
        self._cache = {}
        self._merged: Optional[CSR] = None

    def merged(self) -> CSR:
        """The owned rows' full neighbourhoods in the extended column layout (interior
        columns as they are, halo column j -> ``Lp + j``), built once. With the halo rows
        local, layers 0 and 1 aggregate the owned rows in ONE SpMM pass over it: no second
        (``beta=1``) pass that re-reads and re-writes every row with a halo neighbour.
        Row entries: the interior ones, then the halo ones (fixed order)."""
        if self._merged is None:
            g = self.graph
            it, ht = g.interior, g.halo
            L, Lp = self.L, self.Lp
            dev = it.device
            di, dh = it.degree(), ht.degree()
            rowptr = torch.zeros(L + 1, dtype=torch.long, device=dev)
            torch.cumsum(di + dh, 0, out=rowptr[1:])
            nnz = int(rowptr[-1])
            ncols = self.L1
            col = torch.empty(nnz, dtype=torch.int32 if ncols < 2**31 else torch.int64,
                              device=dev)
            # row chunks of <= ~2^26 entries: bounded int64 temporaries at 1e9+ entries
            step = max(1, int(L * (1 << 26) // max(nnz, 1)))
            for r0 in range(0, L, step):
                r1 = min(L, r0 + step)
                rr = torch.arange(r0, r1, device=dev)
                for part, deg, base, shift in ((it, di, 0, 0), (ht, dh, 1, Lp)):
                    a, b = int(part.rowptr[r0]), int(part.rowptr[r1])
                    if b == a:
                        continue
                    rows = torch.repeat_interleave(rr, deg[r0:r1], output_size=b - a)
                    pos = torch.arange(a, b, device=dev) - part.rowptr[rows] + rowptr[rows]
                    if base:
                        pos += di[rows]
                    col[pos] = (part.col[a:b].long() + shift).to(col.dtype)
                    del rows, pos
            self._merged = CSR(rowptr, col, ncols, None, symmetric=False)
        return self._merged

    def aggregate_owned(self, h_ext: torch.Tensor, out: torch.Tensor,
                        mean: bool = True) -> torch.Tensor:
        """Neighbour mean of the owned rows over an extended-layout input (rows
        ``[0, L)`` owned, ``[Lp, Lp + H)`` halo): one pass over :meth:`merged`."""
        g = self.graph
        m = self.merged()
        g.edges_aggregated += m.nnz
        return K.spmm(m.rowptr, m.col, h_ext, out, row_scale=g.inv_deg if mean else None,
                      split=_hs(m))

    @property
    def nnz(self) -> int:
        return self.csr.nnz

    def inputs(self, x: torch.Tensor) -> torch.Tensor:
        """``[L1 + H2, F]`` first-layer input rows in the extended layout, built once per
        input tensor (weak reference + version: an in-place update rebuilds)."""
        c = self._cache
        if c.get("ref") is not None and c["ref"]() is x and c["version"] == x._version:
            return c["X"]
        c.clear()
        g = self.graph
        X = torch.empty(self.L1 + self.H2, x.shape[1], dtype=x.dtype, device=x.device)
        X[:self.L].copy_(x)
        X[self.L:self.Lp].zero_()
        X[self.Lp:self.L1].copy_(g.a2a(K.gather_rows(x, g.send_map.idx)))
        if self.H2:
            X[self.L1:].copy_(self.a2a2(K.gather_rows(x, self.send_idx2)))
        c.update(ref=weakref.ref(x), version=x._version, X=X)
        return X

    def aggregate0(self, X: torch.Tensor, out: torch.Tensor, mean: bool = True) -> torch.Tensor:
        """First-layer neighbour mean over the ``L1`` extended rows into ``out [L1, F]``:
        owned rows through ``graph`` (halo rows read from ``X``, no exchange), halo rows
        through their own neighbourhood lists."""
        g = self.graph
        L, Lp, L1 = self.L, self.Lp, self.L1
        if MERGED:
            self.aggregate_owned(X, out[:L], mean=mean)
        else:
            g.aggregate(X[:L], mean=mean, out=out[:L], halo_rows=X[Lp:L1])
        if Lp > L:
            out[L:Lp].zero_()
        K.spmm(self.csr.rowptr, self.csr.col, X, out[Lp:L1],
               row_scale=self.inv_deg if mean else None, split=_hs(self.csr))
        g.edges_aggregated += self.csr.nnz
        return out
