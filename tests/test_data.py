"""Data layer: DistributedGraph, renumbering, partitioners, synthetic generator."""
import pytest
import torch

from dgraph_amd.data.graph import DistributedGraph, get_round_robin_node_rank_map
from dgraph_amd.data.partition import label_propagation_partition, partition, partition_stats
from dgraph_amd.data.preprocess import (
    edge_renumbering,
    inverse_permutation,
    node_renumbering,
    process_homogenous_data,
)
from dgraph_amd.data.synthetic import SHAPES, build_local_csr, build_partition, node_data


@pytest.mark.parametrize("n,w,exp", [(0, 3, []), (4, 1, [0, 0, 0, 0]),
                                     (6, 3, [0, 1, 2, 0, 1, 2]), (3, 5, [0, 1, 2])])
def test_round_robin(n, w, exp):
    assert get_round_robin_node_rank_map(n, w).tolist() == exp


def _toy():
    g = torch.Generator().manual_seed(0)
    V = 30
    ei = torch.randint(0, V, (2, 80), generator=g)
    feats = torch.randn(V, 5, generator=g)
    labels = torch.randint(0, 3, (V,), generator=g)
    place = torch.randint(0, 3, (V,), generator=g)
    return V, ei, feats, labels, place


def test_renumbering_preserves_graph():
    V, ei, feats, labels, place = _toy()
    new_to_old, ranks = node_renumbering(place)
    assert (ranks[1:] >= ranks[:-1]).all()
    assert torch.equal(place[new_to_old], ranks)
    e2, sr, dr, _ = edge_renumbering(ei, new_to_old, ranks)
    old_to_new = inverse_permutation(new_to_old)
    # the relabelled edge multiset equals the original one mapped through old_to_new
    a = sorted(map(tuple, old_to_new[ei].t().tolist()))
    b = sorted(map(tuple, e2.t().tolist()))
    assert a == b
    assert (sr[1:] >= sr[:-1]).all()
    assert torch.equal(ranks[e2[0]], sr) and torch.equal(ranks[e2[1]], dr)


def test_process_homogenous_data_and_accessors(tmp_path):
    V, ei, feats, labels, place = _toy()
    split = {"train": torch.arange(0, 10).numpy(), "valid": torch.arange(10, 20).numpy(),
             "test": torch.arange(20, 30).numpy()}
    dg = process_homogenous_data({"node_feat": feats.numpy(), "edge_index": ei.numpy(),
                                  "num_nodes": V, "edge_feat": None},
                                 labels.numpy(), 0, 3, split, place)
    new_to_old, _ = node_renumbering(place)
    assert torch.equal(dg.node_features, feats[new_to_old])
    assert torch.equal(dg.labels, labels[new_to_old])
    # features at both ends of every edge are unchanged by renumbering
    o2n = inverse_permutation(new_to_old)
    assert torch.equal(dg.node_features[o2n[ei[0]]], feats[ei[0]])
    for r in range(3):
        lf = dg.get_local_node_features(r)
        assert lf.shape[0] == int((place == r).sum())
        tr = dg.get_local_mask("train", r)
        start, _ = dg.local_node_range(r)
        assert torch.equal(dg.labels[start + tr], labels[new_to_old][start + tr])
        assert dg.get_local_edge_indices(r).shape[1] == int((dg.edge_loc == r).sum())
    assert dg.get_global_rank_mappings().shape == (2, 80)
    p = tmp_path / "g.pt"
    dg.save(p)
    dg2 = DistributedGraph.load(p)
    assert torch.equal(dg2.edge_index, dg.edge_index) and dg2.world_size == 3


def test_partitioners_and_stats():
    # two 20-vertex cliques joined by one edge: LP from a bad start must find the cut
    a = torch.combinations(torch.arange(20), 2).t()
    b = a + 20
    ei = torch.cat([a, b, torch.tensor([[0], [20]])], 1)
    ei = torch.cat([ei, ei.flip(0)], 1)
    bad = torch.arange(40) % 2
    lp = label_propagation_partition(ei, 40, 2, rounds=20, imbalance=0.1, init=bad)
    s_bad = partition_stats(ei, bad, 2)
    s_lp = partition_stats(ei, lp, 2)
    assert s_lp["edge_cut_frac"] < s_bad["edge_cut_frac"]
    assert s_lp["imbalance"] <= 1.1 + 1e-6
    for m in ("contiguous", "round_robin", "random"):
        p = partition(m, 40, 4)
        assert p.numel() == 40 and int(p.max()) < 4


def test_synthetic_independent_of_world_size():
    shape = SHAPES["ogbn-arxiv"].scaled(0.005)
    csr1, L1, off1 = build_local_csr(shape, 0, 1, "cpu")
    dense_cols = []
    for r in range(3):
        csr, L, off = build_local_csr(shape, r, 3, "cpu")
        dense_cols.append((csr.rowptr, csr.col))
    # concatenated per-rank rows == single-rank rows
    rp = [dense_cols[0][0]]
    cols = torch.cat([c for _, c in dense_cols])
    assert torch.equal(cols.long(), csr1.col.long())
    x1, y1, t1 = node_data(shape, 0, off1, "cpu", dtype=torch.float32)
    xs = torch.cat([node_data(shape, r, off, "cpu", dtype=torch.float32)[0] for r in range(3)])
    _, _, off3 = build_local_csr(shape, 0, 3, "cpu")
    xs = torch.cat([node_data(shape, r, off3, "cpu", dtype=torch.float32)[0] for r in range(3)])
    assert torch.equal(x1, xs)


def test_synthetic_shape_counts():
    shape = SHAPES["ogbn-products"].scaled(0.002)
    p = build_partition(shape, 0, 1, "cpu")
    assert p["csr"].nnz == 2 * shape.num_directed_edges
    assert p["L"] == shape.num_nodes


def _community_graph(k=4, n=25, p_in=0.4, n_bridge=6, seed=0):
    g = torch.Generator().manual_seed(seed)
    es = []
    for c in range(k):
        pairs = torch.combinations(torch.arange(n), 2)
        keep = torch.rand(pairs.shape[0], generator=g) < p_in
        es.append(pairs[keep].t() + c * n)
    es.append(torch.randint(0, k * n, (2, n_bridge), generator=g))
    ei = torch.cat(es, 1)
    return k * n, ei[:, ei[0] != ei[1]]


def _dlp_worker(rank, world, parts):
    import torch.distributed as dist

    from dgraph_amd.data.partition import distributed_label_propagation

    V, ei = _community_graph()
    init = torch.randint(0, parts, (V,), generator=torch.Generator().manual_seed(3))
    # this rank owns adjacency rows [lo, hi) (both directions), global column ids
    lo, hi = rank * V // world, (rank + 1) * V // world
    rows = torch.cat([ei[0], ei[1]])
    cols = torch.cat([ei[1], ei[0]])
    m = (rows >= lo) & (rows < hi)
    r, c = rows[m] - lo, cols[m]
    o = torch.argsort(r * V + c)
    r, c = r[o], c[o]
    rowptr = torch.zeros(hi - lo + 1, dtype=torch.long)
    rowptr[1:] = torch.cumsum(torch.bincount(r, minlength=hi - lo), 0)
    part = distributed_label_propagation(rowptr, c, lo, V, parts, rounds=30, imbalance=0.1,
                                         init=init, seed=1)
    got = [torch.empty_like(part) for _ in range(world)]
    dist.all_gather(got, part)
    assert all(torch.equal(x, part) for x in got), "part vectors diverged across ranks"
    s0 = partition_stats(ei, init, parts, symmetric=True)
    s1 = partition_stats(ei, part, parts, symmetric=True)
    assert s1["edge_cut_frac"] < 0.5 * s0["edge_cut_frac"], (s0["edge_cut_frac"], s1["edge_cut_frac"])
    assert s1["imbalance"] <= 1.1 + 1e-6
    assert s1["halo_rows_total"] < s0["halo_rows_total"]


@pytest.mark.parametrize("world", [1, 2, 4])
def test_distributed_label_propagation(world):
    from conftest import run_ranks

    run_ranks(_dlp_worker, world, 4)


def test_partition_stats_symmetric_matches_concatenated():
    V, ei = _community_graph()
    part = torch.randint(0, 3, (V,), generator=torch.Generator().manual_seed(5))
    a = partition_stats(ei, part, 3, symmetric=True)
    b = partition_stats(torch.cat([ei, ei.flip(0)], 1), part, 3)
    assert a["edge_cut_frac"] == b["edge_cut_frac"]
    assert torch.equal(a["pair_matrix"], b["pair_matrix"])
