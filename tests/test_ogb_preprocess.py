"""OGB preprocessing tool (experiments/OGB/preprocess.py counterpart): networkx pickle
layout, partition + renumbering, placement files, METIS wiring (stand-in module: no
METIS binding is installed, so METIS parity itself is unpinned)."""
import json
import os
import sys
import types

import numpy as np
import torch

from dgraph_amd.experiments import ogb_preprocess as op


def _graph():
    g = torch.Generator().manual_seed(0)
    a = torch.combinations(torch.arange(12), 2).t()
    ei = torch.cat([a, a + 12, a + 24, torch.tensor([[0, 12], [24, 30]])], 1)
    keep = torch.rand(ei.shape[1], generator=g) < 0.6
    return ei[:, keep], 36


def test_networkx_pickle_layout(tmp_path):
    ei, V = _graph()
    p = op.save_networkx_graph(ei.t().numpy(), V, "toy", directed=False, out_dir=str(tmp_path))
    assert os.path.basename(p) == "toy_directed=False.pkl"
    G = op.load_networkx_graph(str(tmp_path / "toy_directed=False"))
    assert G.number_of_nodes() == V and G.number_of_edges() == ei.shape[1]
    p = op.save_networkx_graph(ei, V, "toy", directed=True, out_dir=str(tmp_path))
    G = op.load_networkx_graph(p[:-4])
    assert G.is_directed() and G.number_of_edges() == 2 * ei.shape[1]


def test_partition_graph_renumbers_consistently():
    ei, V = _graph()
    new_to_old, edges, placement = op.partition_graph(ei.t().numpy(), 3, V, method="lp")
    assert placement.shape == (V,) and int(placement.max()) < 3
    # ranks own contiguous blocks in the new numbering
    ranks_new = placement[new_to_old]
    assert bool((ranks_new[1:] >= ranks_new[:-1]).all())
    # relabelled edge multiset == original mapped through old->new
    old_to_new = torch.empty_like(new_to_old)
    old_to_new[new_to_old] = torch.arange(V)
    a = sorted(map(tuple, old_to_new[ei].t().tolist()))
    assert a == sorted(map(tuple, edges.t().tolist()))
    st = op.partition_stats(ei, placement, 3, symmetric=True)
    assert st["edge_cut_frac"] < 0.2 and st["imbalance"] <= 1.06


def test_metis_wiring_with_stand_in(monkeypatch):
    calls = {}
    fake = types.ModuleType("metis")

    def networkx_to_metis(G):
        calls["nodes"] = G.number_of_nodes()
        return G

    def part_graph(G, nparts):
        calls["nparts"] = nparts
        return 0, [v % nparts for v in range(G.number_of_nodes())]

    fake.networkx_to_metis, fake.part_graph = networkx_to_metis, part_graph
    monkeypatch.setitem(sys.modules, "metis", fake)
    assert op.available_methods()[0] == "metis"
    ei, V = _graph()
    _, _, placement = op.partition_graph(ei, 4, V)  # auto -> metis
    assert calls == {"nodes": V, "nparts": 4}
    assert torch.equal(placement, torch.arange(V) % 4)


def test_cli_writes_placement_consumed_by_loaders(tmp_path):
    rc = op.main(["--dset_name", "arxiv", "--num_ranks", "2", "--out_dir", str(tmp_path),
                  "--scale", "0.002", "--method", "lp"])
    assert rc == 0
    assert (tmp_path / "ogbn-arxiv_directed=True.pkl").exists()
    pl = torch.load(tmp_path / "ogbn-arxiv_placement_W2.pt", weights_only=True)
    st = json.loads((tmp_path / "ogbn-arxiv_placement_W2.json").read_text())
    assert pl.numel() == st["num_nodes"] and st["method"] == "lp"
    assert set(np.unique(pl.numpy()).tolist()) <= {0, 1}
