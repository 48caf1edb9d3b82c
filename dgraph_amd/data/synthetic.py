"""Synthetic graphs with the shapes of the OGB datasets named in BASELINE.json.

There is no network (no ogb download), so benchmarks and tests run on generated graphs
of the named size: node count, directed edge count, feature width, class count (SURVEY.md
App. D; the sizes are the public OGB specs). The generator is:

* **deterministic and distributed**: the directed edge list is produced in fixed chunks
  from a seeded counter-based generator; every rank regenerates the chunks and keeps only
  the (symmetrised) entries whose aggregating vertex it owns — no rank ever holds the
  global edge list, and the result is independent of the world size;
* **structured like a real citation graph after partitioning**: a fraction
  ``global_frac`` of edges connects uniformly random endpoints with a hub-skewed
  destination (power-law-like in-degrees, hashed so hubs spread over partitions); the
  rest connect ids within a local window (community structure), so a contiguous vertex
  partition behaves like a METIS partition with a modest edge cut. Both knobs are
  recorded in every benchmark line. ``global_frac=1`` gives a structureless random graph.

Messages are aggregated over the symmetrised graph (each directed pair (u, v) is a
message u->v and v->u), the usual treatment of ogbn-papers100M/products in GNN training.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, asdict
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops.csr import CSR, index_dtype_for


@dataclass(frozen=True)
class GraphShape:
    name: str
    num_nodes: int
    num_directed_edges: int  # pairs before symmetrisation
    num_features: int
    num_classes: int
    train_frac: float
    val_frac: float = 0.0
    test_frac: float = 0.0

    def scaled(self, factor: float) -> "GraphShape":
        return GraphShape(f"{self.name}@{factor:g}", max(int(self.num_nodes * factor), 16),
                          max(int(self.num_directed_edges * factor), 16), self.num_features,
                          self.num_classes, self.train_frac, self.val_frac, self.test_frac)


SHAPES = {
    # OGB public specs (SURVEY.md App. D "External dataset sizes"); split fractions are the
    # official split sizes / num_nodes (arxiv 90,941/29,799/48,603; products
    # 196,615/39,323/2,213,091; papers100M 1,207,179/125,265/214,338)
    "ogbn-arxiv": GraphShape("ogbn-arxiv", 169_343, 1_166_243, 128, 40, 0.537, 0.176, 0.287),
    "ogbn-products": GraphShape("ogbn-products", 2_449_029, 61_859_140, 100, 47, 0.08,
                                0.0161, 0.9037),
    "ogbn-papers100M": GraphShape("ogbn-papers100M", 111_059_956, 1_615_685_872, 128, 172,
                                  0.0109, 0.00113, 0.00193),
    "ogbn-proteins": GraphShape("ogbn-proteins", 132_534, 39_561_252, 8, 112, 0.65, 0.16,
                                0.19),
}


def contiguous_offsets(num_nodes: int, world_size: int) -> List[int]:
    base, rem = divmod(num_nodes, world_size)
    off = [0]
    for r in range(world_size):
        off.append(off[-1] + base + (1 if r < rem else 0))
    return off


_CHUNK = 1 << 26  # directed pairs generated per step (64M)


def _mix(*vals: int) -> int:
    """Deterministic 63-bit seed mixing (splitmix64); Python's hash() of str is salted."""
    h = 0x9E3779B97F4A7C15
    for v in vals:
        h ^= (int(v) + 0x9E3779B97F4A7C15 + ((h << 6) & 0xFFFFFFFFFFFFFFFF) + (h >> 2))
        h &= 0xFFFFFFFFFFFFFFFF
        z = h
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        h = z ^ (z >> 31)
    return h & 0x7FFFFFFFFFFFFFFF


def _chunk_edges(shape: GraphShape, k: int, n: int, seed: int, global_frac: float,
                 window: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
    g = torch.Generator(device=device)
    g.manual_seed(_mix(seed, k))
    V = shape.num_nodes
    src = torch.randint(0, V, (n,), generator=g, device=device, dtype=torch.int64)
    u = torch.rand(n, generator=g, device=device)
    is_global = torch.rand(n, generator=g, device=device) < global_frac
    # global edges: hub-skewed destination (P(rank k) ~ k^-1/2), hashed over the id space
    hub = (u * u * V).long().clamp_(max=V - 1)
    prime = 2_147_483_629  # coprime with any V < 2^31 that is not a multiple of it
    gdst = (hub * prime + 7919) % V
    # local edges: symmetric offset in [-window, window]
    off = ((u * 2 - 1) * window).long()
    ldst = (src + off) % V
    dst = torch.where(is_global, gdst, ldst)
    return src, dst


def build_local_csr(
    shape: GraphShape,
    rank: int,
    world_size: int,
    device,
    seed: int = 0,
    global_frac: float = 0.05,
    window: int = 1 << 14,
    row_buckets: Optional[int] = None,
) -> Tuple[CSR, int, List[int]]:
    """CSR of the symmetrised graph restricted to rows owned by ``rank`` (contiguous
    partition); columns are GLOBAL ids (int64). Returns (csr, num_local, offsets)."""
    off = contiguous_offsets(shape.num_nodes, world_size)
    lo, hi = off[rank], off[rank + 1]
    L = hi - lo
    E = shape.num_directed_edges
    nb = row_buckets or max(1, min(64, (2 * E // world_size) // (1 << 28) + 1))
    bucket_rows = (L + nb - 1) // nb
    buckets_r: List[List[torch.Tensor]] = [[] for _ in range(nb)]
    buckets_c: List[List[torch.Tensor]] = [[] for _ in range(nb)]
    cdt = torch.int32 if shape.num_nodes < 2**31 else torch.int64
    for k in range(0, (E + _CHUNK - 1) // _CHUNK):
        n = min(_CHUNK, E - k * _CHUNK)
        s, d = _chunk_edges(shape, k, n, seed, global_frac, window, device)
        for rows, cols in ((d, s), (s, d)):  # message s->d aggregates at d, and d->s at s
            m = (rows >= lo) & (rows < hi)
            r = (rows[m] - lo)
            c = cols[m]
            b = torch.div(r, bucket_rows, rounding_mode="floor")
            if nb == 1:
                buckets_r[0].append(r.to(torch.int32))
                buckets_c[0].append(c.to(cdt))
            else:
                order = torch.argsort(b, stable=True)
                r, c, b = r[order], c[order], b[order]
                counts = torch.bincount(b, minlength=nb).tolist()
                rs = torch.split(r.to(torch.int32), counts)
                cs = torch.split(c.to(cdt), counts)
                for i in range(nb):
                    if counts[i]:
                        buckets_r[i].append(rs[i])
                        buckets_c[i].append(cs[i])
        del s, d
    deg = torch.zeros(L, dtype=torch.int64, device=device)
    cols_out = []
    for i in range(nb):
        if not buckets_r[i]:
            continue
        r = torch.cat(buckets_r[i]).long()
        c = torch.cat(buckets_c[i])
        buckets_r[i] = buckets_c[i] = None
        key = r * shape.num_nodes + c.long()  # deterministic order: (row, col)
        key, _ = torch.sort(key)
        r = torch.div(key, shape.num_nodes, rounding_mode="floor")
        c = (key - r * shape.num_nodes).to(cdt)
        del key
        deg += torch.bincount(r, minlength=L)
        cols_out.append(c)
        del r
    col = torch.cat(cols_out) if cols_out else torch.zeros(0, dtype=cdt, device=device)
    del cols_out
    rowptr = torch.zeros(L + 1, dtype=torch.int64, device=device)
    torch.cumsum(deg, 0, out=rowptr[1:])
    return CSR(rowptr, col, shape.num_nodes, None, symmetric=False), L, off


def build_rows_csr(shape: GraphShape, row_gids: torch.Tensor, device, seed: int = 0,
                   global_frac: float = 0.05, window: int = 1 << 14) -> CSR:
    """CSR of the symmetrised graph restricted to an arbitrary sorted set of vertices
    ``row_gids`` (e.g. a rank's halo vertices, for halo recomputation); columns are GLOBAL
    ids. The same streaming generator as :func:`build_local_csr`, so each row holds
    exactly the entries (and the (row, col) order) its owner's CSR holds."""
    V = shape.num_nodes
    R = row_gids.numel()
    member = torch.zeros(V, dtype=torch.bool, device=device)
    member[row_gids] = True
    cdt = torch.int32 if V < 2**31 else torch.int64
    keys = []
    E = shape.num_directed_edges
    for k in range(0, (E + _CHUNK - 1) // _CHUNK):
        n = min(_CHUNK, E - k * _CHUNK)
        s_, d_ = _chunk_edges(shape, k, n, seed, global_frac, window, device)
        for rows, cols in ((d_, s_), (s_, d_)):
            m = member[rows]
            r = torch.searchsorted(row_gids, rows[m])
            keys.append(r * V + cols[m])
        del s_, d_
    key = torch.sort(torch.cat(keys)).values if keys else \
        torch.zeros(0, dtype=torch.int64, device=device)
    del keys
    r = torch.div(key, V, rounding_mode="floor")
    col = (key - r * V).to(cdt)
    rowptr = torch.zeros(R + 1, dtype=torch.int64, device=device)
    torch.cumsum(torch.bincount(r, minlength=R), 0, out=rowptr[1:])
    return CSR(rowptr, col, V, None, symmetric=False)


def localize_columns(csr: CSR, rank: int, offsets: List[int]):
    """Relabel global column ids: owned -> [0, L), remote -> L + position in the halo
    (sorted by global id == (owner, id) under contiguous ownership). Returns
    (csr_local, halo_gids, halo_counts_per_owner)."""
    lo, hi = offsets[rank], offsets[rank + 1]
    L = hi - lo
    step = 1 << 28  # chunked: bounded temporaries, no >2^31-element masks
    n = csr.col.numel()
    parts = []
    for a in range(0, n, step):
        c = csr.col[a:a + step].long()
        parts.append(torch.unique(c[(c < lo) | (c >= hi)]))
    halo = torch.unique(torch.cat(parts)) if parts else csr.col.new_zeros(0).long()
    del parts
    H = halo.numel()
    new = torch.empty(n, dtype=index_dtype_for(L + H), device=csr.col.device)
    for a in range(0, n, step):
        c = csr.col[a:a + step].long()
        remote = (c < lo) | (c >= hi)
        loc = c - lo
        if H:
            loc = torch.where(remote, L + torch.searchsorted(halo, c), loc)
        new[a:a + step] = loc.to(new.dtype)
    W = len(offsets) - 1
    off_t = torch.tensor(offsets, device=halo.device, dtype=torch.int64)
    owners = torch.bucketize(halo, off_t, right=True) - 1
    counts = torch.bincount(owners, minlength=W).tolist() if H else [0] * W
    out = CSR(csr.rowptr, new, L + H, None, symmetric=False)
    return out, halo, counts


def _local_send_plan(csr: CSR, L: int, recv_splits: List[int]):
    """For a SYMMETRIC graph: the local rows each peer p receives from this rank (rows with
    an entry in a halo column owned by p), sorted by (p, row), and the per-peer counts."""
    dev = csr.device
    W = len(recv_splits)
    recv_end = torch.cumsum(torch.tensor(recv_splits, dtype=torch.long, device=dev), 0)
    keys = []
    R = csr.num_rows
    nnz = max(csr.col.numel(), 1)
    step = max(1, int(R * (1 << 26) // nnz))
    for r0 in range(0, R, step):
        r1 = min(R, r0 + step)
        a, b = int(csr.rowptr[r0]), int(csr.rowptr[r1])
        if b == a:
            continue
        c = csr.col[a:b].long()
        rows = torch.repeat_interleave(torch.arange(r0, r1, device=dev),
                                       csr.rowptr[r0 + 1:r1 + 1] - csr.rowptr[r0:r1],
                                       output_size=b - a)
        h = c >= L
        owner = torch.searchsorted(recv_end, c[h] - L, right=True)
        keys.append(torch.unique(owner * L + rows[h]))
        del c, rows, h, owner
    key = torch.unique(torch.cat(keys)) if keys else torch.zeros(0, dtype=torch.long,
                                                                 device=dev)
    del keys
    owner = torch.div(key, max(L, 1), rounding_mode="floor")
    send_splits = [int(v) for v in torch.bincount(owner, minlength=W).tolist()]
    send_local_idx = (key - owner * L).to(index_dtype_for(L)).contiguous()
    return send_local_idx, send_splits


def build_partition(shape: GraphShape, rank: int, world_size: int, device, seed: int = 0,
                    global_frac: float = 0.05, window: int = 1 << 14, group=None,
                    rehearse: bool = False):
    """Full per-rank partition: local CSR (local+halo columns) and the halo send plan.

    Returns a dict with keys csr, L, H, halo_gids, send_local_idx, send_splits,
    recv_splits, offsets. Collective over ``group`` when world_size > 1, unless
    ``rehearse``: then rank ``rank`` of a ``world_size``-way partition is built alone, with
    a loopback send plan of the right size (bench.py --rehearse-world).
    """
    from ..plan.pattern import _alltoall_counts, _alltoallv_ids

    csr_g, L, offsets = build_local_csr(shape, rank, world_size, device, seed, global_frac,
                                        window)
    if world_size == 1:  # every column is local already
        csr_g.num_cols = L
        return dict(csr=csr_g, L=L, H=0, halo_gids=csr_g.col[:0].long(),
                    send_local_idx=torch.zeros(0, dtype=torch.int32, device=device),
                    send_splits=[0], recv_splits=[0], offsets=offsets)
    csr, halo, recv_splits = localize_columns(csr_g, rank, offsets)
    del csr_g
    if world_size > 1 and rehearse:
        # one rank of a W-way job in a single process (no peers). The graph is symmetric,
        # so the rows peer p wants from this rank are exactly the local rows with a
        # neighbour owned by p: the real send plan, computed locally (sorted by (p, row),
        # as the peers' requests would be), so every buffer, plan and kernel has its real
        # shape and the interior/boundary split is the real one; the exchange itself is a
        # local loopback (comm/alltoallv.py; link-delayed with DGRAPH_LOOPBACK_LINK_GBPS).
        send_local_idx, send_splits = _local_send_plan(csr, L, recv_splits)
        return dict(csr=csr, L=L, H=int(halo.numel()), halo_gids=halo,
                    send_local_idx=send_local_idx, send_splits=send_splits,
                    recv_splits=recv_splits, offsets=offsets)
    if world_size > 1:
        req = torch.tensor(recv_splits, dtype=torch.long, device=device)
        send_counts = _alltoall_counts(req, group)
        send_splits = [int(v) for v in send_counts.tolist()]
        wanted = _alltoallv_ids(halo, recv_splits, send_splits, group)
        send_local_idx = (wanted - offsets[rank]).to(index_dtype_for(L))
    else:
        send_splits = [0]
        send_local_idx = torch.zeros(0, dtype=torch.int32, device=device)
    return dict(csr=csr, L=L, H=int(halo.numel()), halo_gids=halo,
                send_local_idx=send_local_idx, send_splits=send_splits,
                recv_splits=recv_splits, offsets=offsets)


SPLIT_TRAIN, SPLIT_VALID, SPLIT_TEST, SPLIT_NONE = 0, 1, 2, 3


def node_data(shape: GraphShape, rank: int, offsets: List[int], device, seed: int = 0,
              dtype=torch.bfloat16, return_split: bool = False):
    """Random features [L, F] (dtype), labels [L] and a train mask for owned vertices,
    seeded per global vertex block so results do not depend on the world size.

    ``return_split=True`` returns an int8 split code per vertex instead of the train mask
    (SPLIT_TRAIN / SPLIT_VALID / SPLIT_TEST / SPLIT_NONE at the shape's split fractions;
    the train set is the same as the mask's)."""
    lo, hi = offsets[rank], offsets[rank + 1]
    L = hi - lo
    x = torch.empty(L, shape.num_features, device=device, dtype=dtype)
    y = torch.empty(L, dtype=torch.int64, device=device)
    train = torch.empty(L, dtype=torch.int8 if return_split else torch.bool, device=device)
    tf, vf = shape.train_frac, shape.train_frac + shape.val_frac
    sf = vf + shape.test_frac
    C = 1 << 20  # global vertex chunks: values depend on the vertex id, not on W
    g = torch.Generator(device=device)
    for c in range(lo // C, (hi + C - 1) // C):
        a, b = c * C, min((c + 1) * C, shape.num_nodes)
        g.manual_seed(_mix(seed, 0x6E6F646573, c))
        xc = torch.randn(b - a, shape.num_features, generator=g, device=device)
        yc = torch.randint(0, shape.num_classes, (b - a,), generator=g, device=device)
        u = torch.rand(b - a, generator=g, device=device)
        if return_split:
            tc = torch.full_like(u, SPLIT_NONE, dtype=torch.int8)
            tc[u < sf] = SPLIT_TEST
            tc[u < vf] = SPLIT_VALID
            tc[u < tf] = SPLIT_TRAIN
        else:
            tc = u < tf
        s, e = max(a, lo), min(b, hi)
        x[s - lo:e - lo] = xc[s - a:e - a].to(dtype)
        y[s - lo:e - lo] = yc[s - a:e - a]
        train[s - lo:e - lo] = tc[s - a:e - a]
    return x, y, train
