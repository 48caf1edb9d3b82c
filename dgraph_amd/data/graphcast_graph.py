"""GraphCast static graphs: icosahedral multimesh, grid<->mesh bipartite graphs and their
per-rank partition (experiments/GraphCast/data_utils/*.py behaviour).

* **Multimesh** — a regular icosahedron refined ``mesh_level`` times (every triangle split
  into four, midpoints projected to the unit sphere); the vertices of level ``k`` are a
  prefix of level ``k + 1``'s, so the multimesh is the union of every level's edges on the
  finest vertex set (40 962 vertices, 327 660 directed edges at level 6, as in the
  GraphCast paper; the reference bidirected an already bidirectional edge list and so
  carried every mesh edge twice).
* **grid2mesh** — each grid point sends to its 4 nearest mesh vertices closer than 0.6 x
  the finest mesh's longest edge (k-d tree query instead of a Python loop).
* **mesh2grid** — each grid point receives from the 3 vertices of the finest-mesh face
  whose centroid is nearest.
* Features: node ``[cos lat, sin lon, cos lon]`` (radians); edge ``[dx, dy, dz, |d|] /
  max|d|`` with ``d`` the sender position in the receiver's local frame (rotated so the
  receiver sits at (1, 0, 0)).

**Partition** (``partition="latitude"``, default): grid rows are cut into ``W`` latitude
bands of (nearly) equal size and every mesh vertex goes to the band of its latitude
(mesh counts balanced by latitude quantiles), so halos exist only along band borders.
Edges live with the rank that aggregates them (mesh2mesh: the edge's source — the
processor aggregates at the source, model.py:288-292; grid2mesh: destination mesh vertex;
mesh2grid: destination grid point), so node aggregation is always rank-local and each
edge block needs ONE halo exchange of the other endpoint's features.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..ops.csr import IndexMap
from ..plan.pattern import CommunicationPattern, build_communication_pattern


# ----------------------------------------------------------------------------- geometry
def icosahedron() -> Tuple[np.ndarray, np.ndarray]:
    """12 unit vertices and 20 outward-oriented faces."""
    from scipy.spatial import ConvexHull

    phi = (1.0 + math.sqrt(5.0)) / 2.0
    v = []
    for a in (-1.0, 1.0):
        for b in (-phi, phi):
            v += [(0.0, a, b), (a, b, 0.0), (b, 0.0, a)]
    v = np.asarray(v, dtype=np.float64)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    # GraphCast orientation (data_utils/icosahedral_mesh.py:100-175): rotate about y by
    # (pi - dihedral angle) / 2 so two faces sit symmetric about each pole. The grid2mesh
    # kNN counts depend on it: 1 618 824 edges at level 6 on the 721x1440 grid, as pinned
    # by experiments/GraphCast/tests/test_single_graph_data.py:27.
    ang = (math.pi - 2.0 * math.asin(phi / math.sqrt(3.0))) / 2.0
    c, s = math.cos(ang), math.sin(ang)
    v = v @ np.array([[c, 0.0, -s], [0.0, 1.0, 0.0], [s, 0.0, c]])
    faces = ConvexHull(v).simplices.astype(np.int64)
    # orient counter-clockwise seen from outside
    a, b, c = v[faces[:, 0]], v[faces[:, 1]], v[faces[:, 2]]
    flip = np.einsum("ij,ij->i", np.cross(b - a, c - a), a + b + c) < 0
    faces[flip] = faces[flip][:, [0, 2, 1]]
    return v, faces


def refine(vertices: np.ndarray, faces: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Split every triangle into 4; new (midpoint) vertices are appended."""
    e = np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [2, 0]]])
    e.sort(axis=1)
    uniq, inv = np.unique(e, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    mid = vertices[uniq[:, 0]] + vertices[uniq[:, 1]]
    mid /= np.linalg.norm(mid, axis=1, keepdims=True)
    V = vertices.shape[0]
    F = faces.shape[0]
    ab, bc, ca = (V + inv[:F], V + inv[F:2 * F], V + inv[2 * F:])
    a, b, c = faces[:, 0], faces[:, 1], faces[:, 2]
    new_faces = np.concatenate([np.stack([a, ab, ca], 1), np.stack([b, bc, ab], 1),
                                np.stack([c, ca, bc], 1), np.stack([ab, bc, ca], 1)])
    return np.concatenate([vertices, mid]), new_faces


def mesh_hierarchy(levels: int) -> Tuple[np.ndarray, List[np.ndarray]]:
    """Finest vertices and the face list of every level 0..levels."""
    v, f = icosahedron()
    faces = [f]
    for _ in range(levels):
        v, f = refine(v, f)
        faces.append(f)
    return v, faces


def faces_to_edges(faces: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Directed edges of every face side (both directions for a closed mesh)."""
    src = np.concatenate([faces[:, 0], faces[:, 1], faces[:, 2]])
    dst = np.concatenate([faces[:, 1], faces[:, 2], faces[:, 0]])
    return src, dst


def multimesh_edges(faces_per_level: List[np.ndarray]) -> Tuple[np.ndarray, np.ndarray]:
    src, dst = faces_to_edges(np.concatenate(faces_per_level))
    key = np.unique(src.astype(np.int64) << 32 | dst.astype(np.int64))
    return (key >> 32).astype(np.int64), (key & 0xFFFFFFFF).astype(np.int64)


def xyz_to_latlon(xyz: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    lat = np.arcsin(np.clip(xyz[:, 2], -1.0, 1.0))
    lon = np.arctan2(xyz[:, 1], xyz[:, 0])
    return lat, lon


def latlon_to_xyz(lat_deg: np.ndarray, lon_deg: np.ndarray) -> np.ndarray:
    lat, lon = np.deg2rad(lat_deg), np.deg2rad(lon_deg)
    return np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], 1)


def node_features(xyz: np.ndarray) -> np.ndarray:
    lat, lon = xyz_to_latlon(xyz)
    return np.stack([np.cos(lat), np.sin(lon), np.cos(lon)], 1).astype(np.float32)


def edge_features(src_xyz: np.ndarray, dst_xyz: np.ndarray) -> np.ndarray:
    """Sender position relative to the receiver, in the receiver's local frame."""
    lat, lon = xyz_to_latlon(dst_xyz)
    c1, s1 = np.cos(-lon), np.sin(-lon)
    c2, s2 = np.cos(lat), np.sin(lat)

    def rot(p):
        x = c1 * p[:, 0] - s1 * p[:, 1]
        y = s1 * p[:, 0] + c1 * p[:, 1]
        z = p[:, 2]
        # rotate about y by +lat: brings the receiver to (1, 0, 0)
        return np.stack([c2 * x + s2 * z, y, -s2 * x + c2 * z], 1)

    d = rot(src_xyz) - rot(dst_xyz)
    n = np.linalg.norm(d, axis=1, keepdims=True)
    m = max(float(n.max()), 1e-12) if n.size else 1.0
    return np.concatenate([d / m, n / m], 1).astype(np.float32)


def lat_lon_grid(shape=(721, 1440)) -> Tuple[np.ndarray, np.ndarray]:
    """Grid latitudes (north to south, poles included) and longitudes (0..360)."""
    lat = np.linspace(90.0, -90.0, shape[0])
    lon = np.arange(shape[1]) * (360.0 / shape[1])
    return lat, lon


# ----------------------------------------------------------------------------- global graph
@dataclass
class GlobalGraphCastGraph:
    mesh_xyz: np.ndarray
    grid_xyz: np.ndarray
    grid_shape: Tuple[int, int]
    m2m: Tuple[np.ndarray, np.ndarray]
    g2m: Tuple[np.ndarray, np.ndarray]   # (grid src, mesh dst)
    m2g: Tuple[np.ndarray, np.ndarray]   # (mesh src, grid dst)


def build_global_graph(mesh_level: int = 6, grid_shape=(721, 1440),
                       duplicate_mesh_edges: bool = False) -> GlobalGraphCastGraph:
    """``duplicate_mesh_edges=True`` reproduces the reference's mesh edge list, which
    bidirects the already bidirectional multimesh (``create_graph(to_bidirected=True)``,
    data_utils/graphcast_graph.py:228-233) and so carries every edge twice (655 320 at
    level 6); the default keeps each directed edge once, as in the GraphCast paper."""
    from scipy.spatial import cKDTree

    verts, faces = mesh_hierarchy(mesh_level)
    m_src, m_dst = multimesh_edges(faces)
    if duplicate_mesh_edges:
        m_src, m_dst = np.concatenate([m_src, m_dst]), np.concatenate([m_dst, m_src])
    fs, fd = faces_to_edges(faces[-1])
    max_len = float(np.linalg.norm(verts[fs] - verts[fd], axis=1).max())
    lat, lon = lat_lon_grid(grid_shape)
    LA, LO = np.meshgrid(lat, lon, indexing="ij")
    grid = latlon_to_xyz(LA.reshape(-1), LO.reshape(-1))
    dist, idx = cKDTree(verts).query(grid, k=4)
    keep = dist < 0.6 * max_len
    g_src = np.repeat(np.arange(grid.shape[0]), 4)[keep.reshape(-1)]
    g_dst = idx.reshape(-1)[keep.reshape(-1)]
    fin = faces[-1]
    cent = verts[fin].mean(1)
    _, fidx = cKDTree(cent).query(grid, k=1)
    m2g_src = fin[fidx].reshape(-1)
    m2g_dst = np.repeat(np.arange(grid.shape[0]), 3)
    return GlobalGraphCastGraph(verts, grid, tuple(grid_shape), (m_src, m_dst),
                                (g_src.astype(np.int64), g_dst.astype(np.int64)),
                                (m2g_src.astype(np.int64), m2g_dst.astype(np.int64)))


def latitude_partition(g: GlobalGraphCastGraph, world_size: int
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    """(grid placement, mesh placement) by latitude bands (see module docstring)."""
    H, Wd = g.grid_shape
    rows = torch.tensor_split(torch.arange(H), world_size)
    grid_part = torch.empty(H * Wd, dtype=torch.long)
    for r, rr in enumerate(rows):
        lo, hi = int(rr[0]) if rr.numel() else 0, int(rr[-1]) + 1 if rr.numel() else 0
        grid_part[lo * Wd:hi * Wd] = r
    mlat = np.arcsin(np.clip(g.mesh_xyz[:, 2], -1, 1))
    order = np.argsort(-mlat, kind="stable")  # north to south like the grid
    mesh_part = torch.empty(g.mesh_xyz.shape[0], dtype=torch.long)
    for r, chunk in enumerate(np.array_split(order, world_size)):
        mesh_part[torch.from_numpy(chunk)] = r
    return grid_part, mesh_part


# Work of one rank, per item counted at the rank that aggregates it (grid2mesh edges: the
# mesh destination; mesh2grid: the grid destination; multimesh: the source). Relative
# weights fitted to the per-rank step times of W=8 rehearsals (round 6, `profiles/r06/gc/`,
# after the hub-row split removed the polar ranks' one-row stragglers): a rank step is
# ~10 ms of size-independent cost plus ~4.9e-5 ms per grid point (embedder, encoder grid
# MLP, decoder, final MLP, its 3 mesh2grid edges and ~1.6 grid2mesh edges) and ~1.4e-5 ms
# per multimesh edge (4 processor layers): a grid point weighs ~3.5 multimesh edges.
COST_WEIGHTS = {"grid": 10.0, "mesh": 6.0, "g2m": 1.0, "m2g": 1.0, "m2m": 4.0}


def aligned_latitude_partition(g: GlobalGraphCastGraph, world_size: int,
                               weights: Optional[Dict[str, float]] = None
                               ) -> Tuple[torch.Tensor, torch.Tensor]:
    """(grid placement, mesh placement) with ONE set of latitude cuts for both.

    :func:`latitude_partition` cuts the grid into bands of equal row count (equal latitude
    width) and the mesh into equal-count latitude quantiles (equal AREA). The two sets of
    cuts do not coincide, so a polar rank's mesh band reaches far into its neighbours' grid
    bands: W=8 rank 0 aggregates grid2mesh edges from 108,669 halo grid points (83 % of its
    own 131,040) and holds 2.8x the grid2mesh edges of an equatorial rank. Here grid rows and
    mesh vertices are cut at the same latitudes, placed between grid rows so every band
    carries an equal share of the modelled work (:data:`COST_WEIGHTS`, counted by the
    latitude of each item's aggregating vertex). Edges cross a band only near its borders
    (grid2mesh / mesh2grid reach ~1 degree), so halos are a few grid rows wide."""
    w = dict(COST_WEIGHTS, **(weights or {}))
    H, Wd = g.grid_shape
    lat_rows = np.linspace(90.0, -90.0, H)
    bounds = np.concatenate([[90.0 + 1e-9], (lat_rows[:-1] + lat_rows[1:]) / 2, [-90.0 - 1e-9]])
    mlat = np.degrees(np.arcsin(np.clip(g.mesh_xyz[:, 2], -1, 1)))
    glat = np.repeat(lat_rows, Wd)

    def north(lat: np.ndarray) -> np.ndarray:
        """Items north of every row boundary (latitudes above it)."""
        srt = np.sort(lat)[::-1]
        return np.searchsorted(-srt, -bounds, side="right").astype(np.float64)

    cum = (w["grid"] * np.arange(H + 1) * Wd + w["mesh"] * north(mlat)
           + w["g2m"] * north(mlat[g.g2m[1]]) + w["m2g"] * north(glat[g.m2g[1]])
           + w["m2m"] * north(mlat[g.m2m[0]]))
    total = cum[-1]
    cuts = [0]
    for r in range(1, world_size):
        c = int(np.searchsorted(cum, total * r / world_size))
        if c > 0 and abs(cum[c - 1] - total * r / world_size) < abs(cum[c] - total * r /
                                                                    world_size):
            c -= 1
        cuts.append(int(np.clip(c, cuts[-1] + 1, H - (world_size - r))))
    cuts.append(H)
    grid_part = torch.empty(H * Wd, dtype=torch.long)
    mesh_part = torch.empty(g.mesh_xyz.shape[0], dtype=torch.long)
    for r in range(world_size):
        grid_part[cuts[r] * Wd:cuts[r + 1] * Wd] = r
        sel = (mlat <= bounds[cuts[r]]) & (mlat > bounds[cuts[r + 1]])
        mesh_part[torch.from_numpy(np.nonzero(sel)[0])] = r
    return grid_part, mesh_part


def grid_placement_from_mesh(g: GlobalGraphCastGraph, mesh_part: torch.Tensor) -> torch.Tensor:
    """Grid placement that follows a given mesh placement: every grid vertex goes to the
    owner of the first mesh vertex it is decoded from (its mesh2grid source triangle), so
    the mesh-to-grid edges of a grid vertex stay with one rank and grid halos follow the
    mesh partition boundary."""
    src, dst = g.m2g
    n_grid = g.grid_shape[0] * g.grid_shape[1]
    first = np.full(n_grid, -1, dtype=np.int64)
    # first edge per grid vertex (edges in any order: take the smallest edge index)
    order = np.argsort(dst, kind="stable")
    d_sorted = dst[order]
    starts = np.ones(d_sorted.shape[0], dtype=bool)
    starts[1:] = d_sorted[1:] != d_sorted[:-1]
    first[d_sorted[starts]] = src[order[starts]]
    if (first < 0).any():
        raise ValueError("grid vertex without a mesh2grid edge")
    return mesh_part.long()[torch.from_numpy(first)]


def grid_placement_from_g2m(g: GlobalGraphCastGraph, mesh_part: torch.Tensor) -> torch.Tensor:
    """The reference's grid placement for a given mesh placement
    (experiments/GraphCast/data_utils/graphcast_graph.py:287-324): every grid vertex takes
    the rank of the mesh destination of its grid2mesh edges — edges visited in ascending
    rank order, the last write kept, i.e. the largest such rank — and a grid vertex with no
    grid2mesh edge stays on rank 0. (The reference's loop pairs the rank-sorted edge
    sources with the unsorted edge ranks, :316-322; this is the rule that loop is written
    to implement, with the pairing intact.)"""
    src, dst = g.g2m
    n_grid = g.grid_shape[0] * g.grid_shape[1]
    r = mesh_part.long()[torch.from_numpy(np.asarray(dst, dtype=np.int64))]
    out = torch.zeros(n_grid, dtype=torch.long)
    out.scatter_reduce_(0, torch.from_numpy(np.asarray(src, dtype=np.int64)), r, "amax",
                        include_self=True)
    return out


def load_mesh_placement(path: str, num_mesh: int, world_size: int) -> torch.Tensor:
    """``mesh_vertex_rank_placement.pt`` of the reference (experiments/GraphCast/dataset.py:
    244, microbenchmark_graphcast.py:35): an int tensor [V_mesh] of ranks. Loaded with
    ``weights_only=True`` (no code from the file runs) and validated."""
    t = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(t, torch.Tensor):
        raise ValueError(f"{path}: expected a tensor, got {type(t).__name__}")
    t = t.reshape(-1).long()
    if t.numel() != num_mesh:
        raise ValueError(f"{path}: {t.numel()} entries for a {num_mesh}-vertex mesh")
    if t.numel() and (int(t.min()) < 0 or int(t.max()) >= world_size):
        raise ValueError(f"{path}: ranks outside [0, {world_size})")
    return t


# ----------------------------------------------------------------------------- per rank
@dataclass
class EdgeSet:
    """Edges owned by this rank: ``agg`` (rank-local aggregation vertex) and ``other``
    (index into ``[local | halo]`` rows of the other endpoint's type)."""

    agg: torch.Tensor
    other: torch.Tensor
    num_agg: int
    num_other: int                      # local + halo rows of the other endpoint type
    features: torch.Tensor              # [E, 4]
    pattern: Optional[CommunicationPattern]
    _maps: dict = field(default_factory=dict, repr=False)

    @property
    def num_edges(self) -> int:
        return int(self.agg.numel())

    def agg_map(self) -> IndexMap:
        m = self._maps.get("agg")
        if m is None:
            m = self._maps["agg"] = IndexMap(self.agg, self.num_agg)
        return m

    def other_map(self) -> IndexMap:
        m = self._maps.get("other")
        if m is None:
            m = self._maps["other"] = IndexMap(self.other, self.num_other)
        return m

    def to(self, device) -> "EdgeSet":
        self.agg, self.other = self.agg.to(device), self.other.to(device)
        self.features = self.features.to(device)
        if self.pattern is not None:
            self.pattern = self.pattern.to(device)
        self._maps.clear()
        return self


@dataclass
class DistributedGraphCastGraph:
    rank: int
    world_size: int
    mesh_level: int
    grid_shape: Tuple[int, int]
    grid_global_ids: torch.Tensor        # local grid rows -> global grid id (row-major)
    mesh_global_ids: torch.Tensor        # local mesh rows -> global mesh vertex id
    mesh_node_features: torch.Tensor     # [L_mesh, 3]
    m2m: EdgeSet                         # agg = mesh src (local), other = mesh dst
    g2m: EdgeSet                         # agg = mesh dst (local), other = grid src
    m2g: EdgeSet                         # agg = grid dst (local), other = mesh src

    @property
    def num_local_grid(self) -> int:
        return int(self.grid_global_ids.numel())

    @property
    def num_local_mesh(self) -> int:
        return int(self.mesh_global_ids.numel())

    def to(self, device) -> "DistributedGraphCastGraph":
        self.grid_global_ids = self.grid_global_ids.to(device)
        self.mesh_global_ids = self.mesh_global_ids.to(device)
        self.mesh_node_features = self.mesh_node_features.to(device)
        for es in (self.m2m, self.g2m, self.m2g):
            es.to(device)
        return self


def _edge_set(agg_g: np.ndarray, other_g: np.ndarray, agg_part: torch.Tensor,
              other_part: torch.Tensor, feats: np.ndarray, rank: int, W: int, group,
              bipartite: bool, rehearse: bool = False) -> EdgeSet:
    el = torch.stack([torch.from_numpy(agg_g), torch.from_numpy(other_g)], 1)
    if rehearse and W > 1:
        # one rank of a W-way job in one process: every rank's pattern built in memory
        # (the collectives carried out offline), this rank's kept
        from ..plan.pattern import build_all_patterns_offline

        cp = build_all_patterns_offline(
            el, agg_part, W, neighbor_partitioning=other_part if bipartite else None)[rank]
    else:
        cp = build_communication_pattern(el, agg_part, rank, W,
                                         neighbor_partitioning=other_part if bipartite
                                         else None, group=group)
    mine = (agg_part[el[:, 0]] == rank).numpy()
    lel = cp.local_edge_list
    L_other = int(cp.num_local_neighbor_vertices or cp.num_local_vertices)
    return EdgeSet(lel[:, 0].contiguous(), lel[:, 1].contiguous(), cp.num_local_vertices,
                   L_other + int(cp.num_halo_vertices), torch.from_numpy(feats[mine]),
                   cp if W > 1 else None)


def partition_graphcast_graph(g: GlobalGraphCastGraph, rank: int, world_size: int,
                              grid_part: Optional[torch.Tensor] = None,
                              mesh_part: Optional[torch.Tensor] = None,
                              group=None, grid_rule: str = "g2m",
                              rehearse: bool = False,
                              partition: str = "latitude") -> DistributedGraphCastGraph:
    """Per-rank view (collective when ``world_size > 1``). Local vertices keep increasing
    global-id order. Given only a mesh placement, the grid placement follows it by
    ``grid_rule``: ``"g2m"`` (the reference's: :func:`grid_placement_from_g2m`) or
    ``"m2g"`` (:func:`grid_placement_from_mesh`: decoder edges stay rank-local).
    ``rehearse``: no process group — the patterns of all ranks are built in this process
    and ``rank``'s is kept (a single-GPU rehearsal of one rank of a W-way job).
    ``partition`` (no placement given): ``"latitude"`` (equal grid rows, mesh by latitude
    quantiles) or ``"aligned"`` (:func:`aligned_latitude_partition`: one set of cuts)."""
    if mesh_part is not None and grid_part is None:
        if grid_rule not in ("g2m", "m2g"):
            raise ValueError(f"grid_rule {grid_rule!r}: expected 'g2m' or 'm2g'")
        grid_part = (grid_placement_from_g2m if grid_rule == "g2m"
                     else grid_placement_from_mesh)(g, mesh_part)
    if grid_part is None or mesh_part is None:
        if partition not in ("latitude", "aligned"):
            raise ValueError(f"partition {partition!r}: expected 'latitude' or 'aligned'")
        grid_part, mesh_part = (aligned_latitude_partition if partition == "aligned"
                                else latitude_partition)(g, world_size)
    m_src, m_dst = g.m2m
    g_src, g_dst = g.g2m
    mg_src, mg_dst = g.m2g
    m2m = _edge_set(m_src, m_dst, mesh_part, mesh_part,
                    edge_features(g.mesh_xyz[m_src], g.mesh_xyz[m_dst]), rank, world_size,
                    group, bipartite=False, rehearse=rehearse)
    g2m = _edge_set(g_dst, g_src, mesh_part, grid_part,
                    edge_features(g.grid_xyz[g_src], g.mesh_xyz[g_dst]), rank, world_size,
                    group, bipartite=True, rehearse=rehearse)
    m2g = _edge_set(mg_dst, mg_src, grid_part, mesh_part,
                    edge_features(g.mesh_xyz[mg_src], g.grid_xyz[mg_dst]), rank, world_size,
                    group, bipartite=True, rehearse=rehearse)
    mesh_ids = torch.nonzero(mesh_part == rank).reshape(-1)
    grid_ids = torch.nonzero(grid_part == rank).reshape(-1)
    return DistributedGraphCastGraph(
        rank, world_size, -1, g.grid_shape, grid_ids, mesh_ids,
        torch.from_numpy(node_features(g.mesh_xyz[mesh_ids.numpy()])), m2m, g2m, m2g)
