"""Rank-local vertex renumbering: interior rows first.

The reference renumbers vertices so each rank owns a contiguous id range (I1,
DGraph/data/preprocess.py:6-11) and keeps the original order inside the range; its
RankLocalRenumberingWithMapping (DGraph/distributed/RankLocalOps.py:261-273) only compacts
ids. Inside a rank the order is free, and the MI355X executor uses that freedom: rows with
no halo neighbour and not needed by any peer ("interior" rows) are numbered first,
``[0, L_int)``, the boundary rows after them, ``[L_int, L)``. Then

* a layer's interior rows can be run to completion — aggregation, GEMM, loss, eval —
  while that layer's halo exchange is still on the xGMI links, with no whole-layer
  aggregate buffer (models/sage_fused.py);
* the reverse exchange of the backward only touches boundary rows, so the interior rows'
  input-layer gradient runs while it is in flight.

Each segment keeps the original relative order, so a chunk of consecutive rows still reads
the same neighbourhood window (now two windows, one per segment) and the caches behave as
before; the locality of the ORIGINAL order is measured here, before the permutation, and
kept on the graph as a hint for the SpMM column-pass choice.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..ops.csr import CSR

# entries handled per chunk by the chunked passes (bounded temporaries at 10^9+ entries)
_CHUNK_ENTRIES = 1 << 26


def _row_chunks(rowptr: torch.Tensor, n: int):
    nnz = max(int(rowptr[-1]), 1)
    step = max(1, int(n * _CHUNK_ENTRIES // nnz))
    return [(r0, min(n, r0 + step)) for r0 in range(0, n, step)]


def graph_locality(rowptr: torch.Tensor, col: torch.Tensor, n: int,
                   samples: int = 65536) -> Optional[float]:
    """Fraction of the entries of ``samples`` evenly spaced rows whose column lies within
    +-min(2^16, n/64) (at least 1024) of the row: high on a graph whose neighbour lists stay
    near the row (windowed / METIS-like orders; a narrow SpMM column pass keeps its window
    in the caches), ~0 on a structureless one. ``None`` for an empty graph."""
    if n == 0:
        return None
    dev = rowptr.device
    rows = torch.linspace(0, n - 1, steps=min(n, samples), device=dev).long()
    beg = rowptr[rows]
    deg = (rowptr[rows + 1] - beg).clamp_max(64)
    tot = int(deg.sum())
    if tot == 0:
        return None
    seg = torch.repeat_interleave(torch.arange(rows.numel(), device=dev), deg)
    off = torch.cumsum(deg, 0) - deg
    pos = beg[seg] + (torch.arange(tot, device=dev) - off[seg])
    dist_ = (col[pos].long() - rows[seg]).abs()
    win = max(1024, min(1 << 16, n // 64))
    return float((dist_ < win).float().mean())


def boundary_mask(csr: CSR, L: int, send_local_idx: Optional[torch.Tensor]) -> torch.Tensor:
    """bool [L]: row has an entry in a halo column (>= L) or is sent to a peer."""
    dev = csr.device
    halo_deg = torch.zeros(L, dtype=torch.long, device=dev)
    for r0, r1 in _row_chunks(csr.rowptr, L):
        a, b = int(csr.rowptr[r0]), int(csr.rowptr[r1])
        if b == a:
            continue
        h = csr.col[a:b] >= L
        rows = torch.repeat_interleave(torch.arange(r0, r1, device=dev),
                                       csr.rowptr[r0 + 1:r1 + 1] - csr.rowptr[r0:r1],
                                       output_size=b - a)
        halo_deg[r0:r1] = torch.bincount(rows[h] - r0, minlength=r1 - r0)
        del h, rows
    bnd = halo_deg > 0
    if send_local_idx is not None and send_local_idx.numel():
        bnd[send_local_idx.long()] = True
    return bnd


def permute_local_rows(csr: CSR, perm: torch.Tensor, inv: torch.Tensor, L: int) -> CSR:
    """Row ``i`` of the result is row ``perm[i]`` of ``csr`` (entry order kept), local
    columns ``c < L`` relabelled ``inv[c]``, halo columns unchanged. Chunked."""
    dev = csr.device
    deg_new = (csr.rowptr[1:] - csr.rowptr[:-1])[perm]
    rowptr = torch.zeros(L + 1, dtype=torch.long, device=dev)
    torch.cumsum(deg_new, 0, out=rowptr[1:])
    col = torch.empty_like(csr.col)
    inv_c = inv.to(csr.col.dtype)
    for r0, r1 in _row_chunks(rowptr, L):
        a, b = int(rowptr[r0]), int(rowptr[r1])
        if b == a:
            continue
        shift = torch.repeat_interleave(csr.rowptr[perm[r0:r1]] - rowptr[r0:r1],
                                        deg_new[r0:r1], output_size=b - a)
        src = torch.arange(a, b, device=dev, dtype=torch.long).add_(shift)
        del shift
        c = csr.col[src]
        del src
        loc = c < L
        col[a:b] = torch.where(loc, inv_c[c.long().clamp_max(L - 1)], c)
        del c, loc
    out = CSR(rowptr, col, csr.num_cols, None, symmetric=csr.symmetric)
    return out


def interior_first(csr: CSR, L: int, send_local_idx: Optional[torch.Tensor]
                   ) -> Tuple[CSR, torch.Tensor, torch.Tensor, int, Optional[float]]:
    """Renumber a rank's rows interior-first. ``csr``: the rank's local CSR (rows = its L
    vertices, columns ``[0, L)`` local and ``[L, L + H)`` halo). Returns ``(csr_new,
    send_local_idx_new, perm, L_int, locality)``: row ``i`` of the new numbering is old row
    ``perm[i]`` (apply ``x = x[perm]`` to every per-vertex tensor), the first ``L_int`` rows
    are interior, ``locality`` is :func:`graph_locality` of the original order."""
    loc = graph_locality(csr.rowptr, csr.col, L)
    bnd = boundary_mask(csr, L, send_local_idx)
    perm = torch.cat([torch.nonzero(~bnd).reshape(-1), torch.nonzero(bnd).reshape(-1)])
    L_int = L - int(bnd.sum())
    del bnd
    inv = torch.empty(L, dtype=torch.long, device=csr.device)
    inv[perm] = torch.arange(L, device=csr.device)
    new = permute_local_rows(csr, perm, inv, L)
    send_new = None
    if send_local_idx is not None:
        send_new = inv[send_local_idx.long()].to(send_local_idx.dtype).contiguous()
    return new, send_new, perm, L_int, loc
