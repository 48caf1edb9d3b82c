"""CommunicationPattern / compute_* helpers.

Same literal graphs and expectations as the reference's tests/test_comm_info.py
(homogeneous 4-vertex / 2-rank graph; bipartite 3x4 graph), single-process tests for
the pure functions, and gloo multi-process tests for the collective builders (the
reference needed 2 GPUs + torchrun for those).
"""
import pytest
import torch
import torch.distributed as dist

from dgraph_amd.plan.pattern import (
    CommunicationPattern,
    build_communication_pattern,
    compute_boundary_vertices,
    compute_comm_map,
    compute_halo_vertices,
    compute_local_edge_list,
    compute_local_vertices,
    compute_recv_offsets,
)

HOMO_EDGE_LIST = torch.tensor([[0, 1], [1, 0], [0, 2], [2, 0], [1, 3], [3, 1], [2, 3], [3, 2]])
HOMO_PARTITIONING = torch.tensor([0, 0, 1, 1])
HETERO_EDGE_LIST = torch.tensor([[0, 0], [0, 2], [1, 1], [1, 3], [2, 0], [2, 2]])
HETERO_SRC_PARTITIONING = torch.tensor([0, 0, 1])
HETERO_DST_PARTITIONING = torch.tensor([0, 0, 1, 1])
HOMO_COMM_MAP = torch.tensor([[0, 2], [2, 0]])


@pytest.mark.parametrize("rank,expected", [(0, [0, 1]), (1, [2, 3])])
def test_local_vertices(rank, expected):
    assert compute_local_vertices(HOMO_PARTITIONING, rank).tolist() == expected


def test_local_vertices_cover_all():
    allv = torch.cat([compute_local_vertices(HOMO_PARTITIONING, r) for r in (0, 1)])
    assert sorted(allv.tolist()) == [0, 1, 2, 3]


@pytest.mark.parametrize("rank,expected", [(0, [2, 3]), (1, [0, 1])])
def test_halo_homogeneous(rank, expected):
    assert compute_halo_vertices(HOMO_EDGE_LIST, HOMO_PARTITIONING, rank).tolist() == expected


def test_halo_empty_and_unique():
    el = torch.tensor([[0, 1], [1, 0]])
    assert compute_halo_vertices(el, torch.tensor([0, 0]), 0).numel() == 0
    el = torch.tensor([[0, 2], [0, 2], [1, 2]])
    assert compute_halo_vertices(el, torch.tensor([0, 0, 1, 1]), 0).tolist() == [2]


@pytest.mark.parametrize("rank,expected", [(0, [2, 3]), (1, [0])])
def test_halo_heterogeneous(rank, expected):
    h = compute_halo_vertices(HETERO_EDGE_LIST, HETERO_SRC_PARTITIONING, rank,
                              dst_partitioning=HETERO_DST_PARTITIONING)
    assert h.tolist() == expected
    assert (HETERO_DST_PARTITIONING[h] != rank).all()


@pytest.mark.parametrize("rank", [0, 1])
def test_local_edge_list(rank):
    lv = compute_local_vertices(HOMO_PARTITIONING, rank)
    hv = compute_halo_vertices(HOMO_EDGE_LIST, HOMO_PARTITIONING, rank)
    le = compute_local_edge_list(HOMO_EDGE_LIST, HOMO_PARTITIONING, lv, hv, rank)
    assert set(map(tuple, le.tolist())) == {(0, 1), (1, 0), (0, 2), (1, 3)}
    assert (le[:, 0] < 2).all() and (le >= 0).all() and (le < 4).all()


@pytest.mark.parametrize("rank,expected", [(0, [0, 0, 2]), (1, [0, 2, 2])])
def test_boundary_homogeneous(rank, expected):
    lv = compute_local_vertices(HOMO_PARTITIONING, rank)
    idx, off = compute_boundary_vertices(HOMO_EDGE_LIST, HOMO_PARTITIONING, lv, rank, 2)
    assert off.tolist() == expected
    assert (idx >= 0).all() and (idx < lv.numel()).all()
    for p in range(2):
        seg = idx[off[p]:off[p + 1]]
        assert seg.unique().numel() == seg.numel()
    assert off[rank + 1] == off[rank]


def test_boundary_dedup_and_empty():
    el = torch.tensor([[0, 2], [0, 2], [0, 3]])
    part = torch.tensor([0, 0, 1, 1])
    idx, off = compute_boundary_vertices(el, part, torch.tensor([0, 1]), 0, 2)
    assert (idx == 0).sum() == 1
    el = torch.tensor([[0, 1], [1, 0]])
    idx, off = compute_boundary_vertices(el, torch.tensor([0, 0]), torch.tensor([0, 1]), 0, 2)
    assert idx.numel() == 0 and off.tolist() == [0, 0, 0]


@pytest.mark.parametrize("rank,expected,n", [(0, [0, 0, 2], 2), (1, [0, 1, 1], 1)])
def test_boundary_heterogeneous(rank, expected, n):
    lv = compute_local_vertices(HETERO_SRC_PARTITIONING, rank)
    idx, off = compute_boundary_vertices(HETERO_EDGE_LIST, HETERO_SRC_PARTITIONING, lv, rank,
                                         2, dst_partitioning=HETERO_DST_PARTITIONING)
    assert off.tolist() == expected and idx.numel() == n


@pytest.mark.parametrize("rank,expected,bwd", [(0, [0, 0, 2], [0, 0]), (1, [0, 2, 2], [0, 2])])
def test_recv_offsets(rank, expected, bwd):
    ro, rb = compute_recv_offsets(HOMO_COMM_MAP, rank)
    assert ro.tolist() == expected
    assert rb.tolist() == bwd
    assert (ro[1:] >= ro[:-1]).all()
    # D11: comm_map dtype contract is integer; float maps are accepted too
    ro2, _ = compute_recv_offsets(HOMO_COMM_MAP.float(), rank)
    assert ro2.tolist() == expected


# ----------------------------------------------------------------------------- gloo W=2
def _dist_homo(rank, world):
    cp = build_communication_pattern(HOMO_EDGE_LIST, HOMO_PARTITIONING, rank, world)
    assert cp.num_local_vertices == 2 and cp.num_halo_vertices == 2
    assert cp.comm_map.tolist() == [[0, 2], [2, 0]]
    exp = {0: [0, 0, 2], 1: [0, 2, 2]}
    assert cp.send_offset.tolist() == exp[rank]
    assert cp.recv_offset.tolist() == exp[rank]
    assert torch.equal(cp.put_forward_remote_offset, cp.comm_map[:rank, :].sum(0))
    assert torch.equal(cp.put_backward_remote_offset, cp.comm_map[:, :rank].sum(1))
    assert set(map(tuple, cp.local_edge_list.tolist())) == {(0, 1), (1, 0), (0, 2), (1, 3)}
    assert cp.comm_map[rank].sum() == cp.send_offset[-1]
    assert cp.comm_map[:, rank].sum() == cp.recv_offset[-1]
    # row of comm_map == my send counts; all-gather symmetry
    sc = cp.send_offset[1:] - cp.send_offset[:-1]
    assert torch.equal(cp.comm_map[rank], sc)
    cm = compute_comm_map(cp.send_offset, world)
    assert torch.equal(cm, cp.comm_map)


def test_build_pattern_homogeneous_w2(ranks):
    ranks(_dist_homo, 2)


def _dist_hetero(rank, world):
    lv = compute_local_vertices(HETERO_SRC_PARTITIONING, rank)
    halo = compute_halo_vertices(HETERO_EDGE_LIST, HETERO_SRC_PARTITIONING, rank,
                                 HETERO_DST_PARTITIONING)
    idx, off = compute_boundary_vertices(HETERO_EDGE_LIST, HETERO_SRC_PARTITIONING, lv, rank,
                                         world, HETERO_DST_PARTITIONING)
    comm = compute_comm_map(off, world)
    ro, _ = compute_recv_offsets(comm, rank)
    assert lv.numel() == {0: 2, 1: 1}[rank] and halo.numel() == {0: 2, 1: 1}[rank]
    assert off.tolist() == {0: [0, 0, 2], 1: [0, 1, 1]}[rank]
    assert ro.tolist() == {0: [0, 0, 1], 1: [0, 2, 2]}[rank]
    assert comm.tolist() == [[0, 2], [1, 0]]


def test_hetero_halo_and_boundary_w2(ranks):
    ranks(_dist_hetero, 2)


def _random_pattern_exchange(rank, world, symmetric):
    from dgraph_amd.comm.alltoallv import AllToAllV

    g = torch.Generator().manual_seed(1)
    V = 40
    E = torch.randint(0, V, (200, 2), generator=g)
    if symmetric:
        E = torch.cat([E, E.flip(1)])
    part = torch.randint(0, world, (V,), generator=g)  # non-contiguous placement
    cp = build_communication_pattern(E, part, rank, world)
    X = torch.randn(V, 5, generator=g)
    lv = cp.local_vertices
    x_local = X[lv]
    a2a = AllToAllV(cp.send_splits(), cp.recv_splits())
    halo_feats = a2a(x_local[cp.send_local_idx])
    # halo rows are in receive order and match their global ids
    assert torch.equal(halo_feats, X[cp.halo_vertices])
    sub = torch.cat([x_local, halo_feats])
    mine = E[part[E[:, 0]] == rank]
    le = cp.local_edge_list
    assert torch.equal(sub[le[:, 1]], X[mine[:, 1]])
    assert torch.equal(lv[le[:, 0]], mine[:, 0])


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("symmetric", [True, False])
def test_pattern_any_partition_any_graph(ranks, world, symmetric):
    """Request-based builder is correct for round-robin/random placements and for
    NON-symmetric graphs (the reference's halo order is only right for symmetric graphs
    under contiguous ownership)."""
    ranks(_random_pattern_exchange, world, symmetric)


def _bipartite(rank, world):
    from dgraph_amd.comm.alltoallv import AllToAllV

    g = torch.Generator().manual_seed(2)
    Vc, Vn = 30, 50
    E = torch.stack([torch.randint(0, Vc, (150,), generator=g),
                     torch.randint(0, Vn, (150,), generator=g)], 1)
    pc = torch.randint(0, world, (Vc,), generator=g)
    pn = torch.randint(0, world, (Vn,), generator=g)
    cp = build_communication_pattern(E, pc, rank, world, neighbor_partitioning=pn)
    Xn = torch.randn(Vn, 3, generator=g)
    ln = compute_local_vertices(pn, rank)
    halo = AllToAllV(cp.send_splits(), cp.recv_splits())(Xn[ln][cp.send_local_idx])
    sub = torch.cat([Xn[ln], halo])
    mine = E[pc[E[:, 0]] == rank]
    assert torch.equal(sub[cp.local_edge_list[:, 1]], Xn[mine[:, 1]])


def test_bipartite_neighbor_partitioning(ranks):
    """D5: the GraphCast call with neighbor_partitioning= works."""
    ranks(_bipartite, 3)


def test_single_rank_pattern():
    cp = build_communication_pattern(HOMO_EDGE_LIST, torch.zeros(4, dtype=torch.long), 0, 1)
    assert cp.num_halo_vertices == 0 and cp.send_local_idx.numel() == 0
    assert cp.local_edge_list.shape == (8, 2)
    assert cp.stats()["num_local"] == 4
