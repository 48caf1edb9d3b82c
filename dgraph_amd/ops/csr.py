"""Compressed-sparse-row graph storage (destination-major) and its transpose.

Every aggregation in dgraph_amd is a CSR SpMM over destination rows, which makes the
local scatter-sum of the reference (``scatter_add`` at GCN.py:57-65, K7/K8 atomics at
local_data_kernels.cuh:301-406) deterministic and atomic-free. A CSR is built once per
plan (plans are static, reference invariant I6) and its transpose — needed for the
backward pass — is built lazily and cached.

Index width: columns are int32 whenever the column space is < 2^31 (half the bytes of
the reference's int64 indices); row pointers are always int64 (papers100M-shaped
graphs have > 2^31 symmetric edges).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import torch

INT32_MAX = 2**31 - 1


def index_dtype_for(n: int) -> torch.dtype:
    return torch.int32 if n <= INT32_MAX else torch.int64


def _rowptr_from_sorted_rows(rows_sorted: torch.Tensor, num_rows: int) -> torch.Tensor:
    counts = torch.bincount(rows_sorted, minlength=num_rows) if rows_sorted.numel() else \
        torch.zeros(num_rows, dtype=torch.long, device=rows_sorted.device)
    rowptr = torch.zeros(num_rows + 1, dtype=torch.long, device=rows_sorted.device)
    torch.cumsum(counts, 0, out=rowptr[1:])
    return rowptr


@dataclass(frozen=True)
class HubSplit:
    """Hub-row split of a CSR (see :meth:`CSR.hub_split`): ``hub_rows[h]`` owns segments
    ``hub_seg_ptr[h] .. hub_seg_ptr[h+1]``; segment ``i`` is ``col[seg_beg[i]:seg_end[i]]``."""

    cap: int
    hub_rows: torch.Tensor
    hub_seg_ptr: torch.Tensor
    seg_beg: torch.Tensor
    seg_end: torch.Tensor

    @property
    def num_segments(self) -> int:
        return self.seg_beg.numel()


@dataclass
class CSR:
    """A sparse [num_rows, num_cols] pattern in CSR form.

    ``perm[k]`` is the index of CSR slot ``k`` in the edge order it was built from
    (``None`` when the input was already destination-sorted). Edge-valued tensors given in
    the original order are permuted with it once (``csr.permute_edges``).
    """

    rowptr: torch.Tensor
    col: torch.Tensor
    num_cols: int
    perm: Optional[torch.Tensor] = None
    symmetric: bool = False
    _transpose: Optional["CSR"] = field(default=None, repr=False)
    _inv_deg: Optional[torch.Tensor] = field(default=None, repr=False)
    _hub: Optional[tuple] = field(default=None, repr=False)
    # row-compacted CSR (see compact_rows): CSR row r is output row row_map[r]
    row_map: Optional[torch.Tensor] = None
    _compact: Optional["CSR"] = field(default=None, repr=False)

    @property
    def num_rows(self) -> int:
        return self.rowptr.numel() - 1

    @property
    def nnz(self) -> int:
        return self.col.numel()

    @property
    def device(self) -> torch.device:
        return self.rowptr.device

    def degree(self) -> torch.Tensor:
        return self.rowptr[1:] - self.rowptr[:-1]

    def inv_degree(self) -> torch.Tensor:
        """fp32 ``1/max(deg,1)`` (mean-aggregation row scale), cached."""
        if self._inv_deg is None:
            self._inv_deg = (1.0 / self.degree().clamp(min=1).float()).contiguous()
        return self._inv_deg

    def hub_split(self, cap: int) -> Optional["HubSplit"]:
        """Hub-row split for the native SpMM (cached per ``cap``): rows with more than
        ``cap`` entries keep their first ``cap`` in the main pass; their tails are cut into
        segments of at most ``cap`` entries (ranges of THIS csr's ``col``, no copy) that are
        summed as independent waves and added back in segment order. ``None`` when no row
        exceeds ``cap`` (or ``cap <= 0``)."""
        if cap <= 0:
            return None
        if self._hub is not None and self._hub[0] == cap:
            return self._hub[1]
        deg = self.degree()
        hub_rows = torch.nonzero(deg > cap).reshape(-1)
        split = None
        if hub_rows.numel() > 0:
            nh = hub_rows.numel()
            tail = deg[hub_rows] - cap
            nseg = torch.div(tail + cap - 1, cap, rounding_mode="floor")
            seg_ptr = torch.zeros(nh + 1, dtype=torch.long, device=self.device)
            torch.cumsum(nseg, 0, out=seg_ptr[1:])
            S = int(seg_ptr[-1].item())
            seg_hub = torch.repeat_interleave(torch.arange(nh, device=self.device), nseg,
                                              output_size=S)
            k = torch.arange(S, device=self.device) - seg_ptr[seg_hub]
            start = self.rowptr[hub_rows][seg_hub]
            beg = start + cap + k * cap
            end = torch.minimum(beg + cap, self.rowptr[hub_rows + 1][seg_hub])
            out_rows = hub_rows if self.row_map is None else self.row_map[hub_rows]
            split = HubSplit(int(cap), out_rows.contiguous(), seg_ptr, beg.contiguous(),
                             end.contiguous())
        self._hub = (cap, split)
        return split

    def compact_rows(self) -> "CSR":
        """The same entries over the non-empty rows only, with ``row_map`` giving each
        row's output row (cached). For the halo / segment-sum blocks of a partition, where
        a pass with ``beta=1`` would otherwise read and rewrite every output row, also the
        ~30-60 % with no entry. The ``col`` array is shared (no copy)."""
        if self.row_map is not None:
            return self
        if self._compact is None:
            nz = torch.nonzero(self.degree() > 0).reshape(-1)
            rowptr = torch.cat([self.rowptr[nz], self.rowptr[-1:]]).contiguous()
            self._compact = CSR(rowptr, self.col, self.num_cols, self.perm, False, None, None,
                                row_map=nz.contiguous())
        return self._compact

    def row_ids(self) -> torch.Tensor:
        return torch.repeat_interleave(
            torch.arange(self.num_rows, device=self.device), self.degree()
        )

    def permute_edges(self, edge_values: torch.Tensor) -> torch.Tensor:
        return edge_values if self.perm is None else edge_values[self.perm]

    def _moved(self, device) -> "CSR":
        return CSR(
            self.rowptr.to(device),
            self.col.to(device),
            self.num_cols,
            None if self.perm is None else self.perm.to(device),
            self.symmetric,
            None,
            None if self._inv_deg is None else self._inv_deg.to(device),
            row_map=None if self.row_map is None else self.row_map.to(device),
        )

    def to(self, device) -> "CSR":
        """Move to ``device``, keeping the cached transpose (and its back link)."""
        new = self._moved(device)
        t = self._transpose
        if t is self:
            new._transpose = new
        elif t is not None:
            nt = t._moved(device)
            nt._transpose = new
            new._transpose = nt
        return new

    @staticmethod
    def from_coo(
        rows: torch.Tensor,
        cols: torch.Tensor,
        num_rows: int,
        num_cols: int,
        *,
        index_dtype: Optional[torch.dtype] = None,
        keep_perm: bool = True,
    ) -> "CSR":
        """Build from COO pairs (row = destination / aggregation target)."""
        rows = rows.reshape(-1)
        cols = cols.reshape(-1)
        idt = index_dtype or index_dtype_for(num_cols)
        if rows.numel() == 0:
            return CSR(
                torch.zeros(num_rows + 1, dtype=torch.long, device=rows.device),
                torch.zeros(0, dtype=idt, device=rows.device),
                num_cols,
                torch.zeros(0, dtype=torch.long, device=rows.device) if keep_perm else None,
            )
        sorted_already = bool((rows[1:] >= rows[:-1]).all()) if rows.numel() > 1 else True
        if sorted_already:
            perm = None
            rs, cs = rows, cols
        else:
            rs, perm = torch.sort(rows, stable=True)
            cs = cols[perm]
        rowptr = _rowptr_from_sorted_rows(rs.long(), num_rows)
        return CSR(rowptr, cs.to(idt).contiguous(), num_cols,
                   perm if keep_perm else None)

    def transpose(self) -> "CSR":
        """CSR of the transposed pattern; ``perm`` maps its slots to THIS CSR's slots."""
        if self._transpose is None:
            if self.symmetric:
                # Same structure; slot k of A^T is slot k of A only as a pattern.
                self._transpose = self
            else:
                cols = self.col.long()
                ct, perm = torch.sort(cols, stable=True)
                rows = self.row_ids()[perm]
                rowptr = _rowptr_from_sorted_rows(ct, self.num_cols)
                t = CSR(rowptr, rows.to(index_dtype_for(self.num_rows)).contiguous(),
                        self.num_rows, perm)
                t._transpose = self
                self._transpose = t
        return self._transpose

    def select_rows(self, rows: torch.Tensor) -> "CSR":
        """CSR of the row subset ``rows`` (in that order; columns unchanged). Used for the
        output layer's gradient, which is nonzero only on the loss rows: A[rows, :]^T
        touches ~|rows| x avg-degree entries instead of every edge."""
        rows = rows.long()
        deg = self.degree()[rows]
        rowptr = torch.zeros(rows.numel() + 1, dtype=torch.long, device=self.device)
        torch.cumsum(deg, 0, out=rowptr[1:])
        nnz = int(rowptr[-1].item())
        if nnz == 0:
            return CSR(rowptr, self.col[:0].clone(), self.num_cols)
        # slot k of new row j reads old slot rowptr[rows[j]] + (k - rowptr_new[j])
        shift = torch.repeat_interleave(self.rowptr[rows] - rowptr[:-1], deg,
                                        output_size=nnz)
        src = torch.arange(nnz, device=self.device, dtype=torch.long).add_(shift)
        return CSR(rowptr, self.col[src].contiguous(), self.num_cols)

    def split_columns(self, boundary: int) -> tuple["CSR", "CSR"]:
        """Split into (cols < boundary) and (cols >= boundary, shifted by -boundary).

        Used for interior/halo overlap: the interior part runs while the halo
        all-to-all-v is in flight. Both parts keep every row (empty rows allowed).
        """
        col = self.col.long()
        is_int = col < boundary
        rows = self.row_ids()
        parts = []
        for mask, shift, ncols in ((is_int, 0, boundary), (~is_int, boundary, self.num_cols - boundary)):
            r = rows[mask]
            c = col[mask] - shift
            rowptr = _rowptr_from_sorted_rows(r, self.num_rows)
            # slot -> original-edge map only when the parent keeps one (edge features)
            base_perm = None if self.perm is None else self.perm[mask]
            parts.append(CSR(rowptr, c.to(index_dtype_for(max(ncols, 1))).contiguous(),
                             ncols, base_perm))
        return parts[0], parts[1]

    def memory_bytes(self) -> int:
        n = self.rowptr.numel() * 8 + self.col.numel() * self.col.element_size()
        if self.perm is not None:
            n += self.perm.numel() * 8
        return n


class IndexMap:
    """A static index vector ``idx`` into ``num_src`` rows, with a cached deterministic
    transpose (a CSR of slot lists per source row) so ``index_add`` / gather-backward
    runs as an atomic-free segment sum instead of float atomics (I4/I5 plans are static).
    """

    def __init__(self, idx: torch.Tensor, num_src: int):
        self.idx = idx.contiguous()
        self.num_src = int(num_src)
        self._t: Optional[CSR] = None

    def to(self, device) -> "IndexMap":
        m = IndexMap(self.idx.to(device), self.num_src)
        if self._t is not None:
            m._t = self._t.to(device)
        return m

    def transpose_csr(self) -> CSR:
        """Rows = source rows, columns = slots ``i`` with ``idx[i] == row``."""
        if self._t is None:
            n = self.idx.numel()
            slots = torch.arange(n, device=self.idx.device)
            self._t = CSR.from_coo(self.idx.long(), slots, self.num_src, n, keep_perm=False)
        return self._t

    # Hub cap of the transposed segment sums. GraphCast's maps are the case it is for: a
    # polar mesh vertex receives 3,753 grid2mesh edges and feeds 6,157 mesh2grid edges
    # (means 40 and 76); unsplit, the one wave holding that row outlasts the rest of a W=8
    # rank's kernel.
    HUB_CAP = 256

    def transpose_split(self) -> Optional[HubSplit]:
        """:meth:`CSR.hub_split` of :meth:`transpose_csr` at :data:`HUB_CAP` (None when no
        source row has more slots), for ``K.spmm(..., split=...)``."""
        return self.transpose_csr().hub_split(self.HUB_CAP)
