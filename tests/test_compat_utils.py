"""CPU tests: the ``DGraph`` API-compatibility tree, torch_local / RankLocalOps
equivalents, the OGB dataset wrapper (synthetic fallback) and the utils subsystem
(TimingReport, RunConfig, checkpoint/resume)."""
import importlib
import os
import pkgutil

import pytest
import torch

from conftest import REPO, run_ranks


# --------------------------------------------------------------------------- DGraph shim
def _dgraph_modules():
    import DGraph

    names = ["DGraph"]
    for m in pkgutil.walk_packages(DGraph.__path__, "DGraph."):
        names.append(m.name)
    return names


def test_dgraph_tree_imports():
    names = _dgraph_modules()
    assert len(names) >= 25
    for n in names:
        importlib.import_module(n)


def test_dgraph_reference_names():
    from DGraph.Communicator import Communicator
    from DGraph.distributed.nccl import COO_to_NCCLCommPlan, NCCLGraphCommPlan
    from DGraph.distributed.haloExchange import HaloExchange, DGraphMessagePassing
    from DGraph.distributed.commInfo import CommunicationPattern, build_communication_pattern
    from DGraph.torch_local import (local_masked_gather, local_masked_scatter,
                                    local_masked_scatter_gather,
                                    local_masked_scatter_add_gather)
    from DGraph.torch_nvshmem_p2p import NVSHMEMP2P
    from DGraph.data.ogbn_datasets import DistributedOGBWrapper
    from DGraph.utils.TimingReport import TimingReport

    assert Communicator is not None and callable(COO_to_NCCLCommPlan)
    for fn in (local_masked_gather, local_masked_scatter, local_masked_scatter_gather,
               local_masked_scatter_add_gather):
        assert callable(fn)
    assert hasattr(NVSHMEMP2P, "dist_get") and hasattr(DistributedOGBWrapper, "__getitem__")
    assert hasattr(TimingReport, "report")
    del NCCLGraphCommPlan, HaloExchange, DGraphMessagePassing, CommunicationPattern
    del build_communication_pattern


# --------------------------------------------------------------------------- torch_local
def test_local_masked_gather_and_scatter_cpu():
    from dgraph_amd.ops import local as L

    torch.manual_seed(0)
    B, N, F, E, R = 2, 30, 8, 50, 20
    x = torch.randn(B, N, F)
    idx = torch.randint(0, N, (E,))
    place = torch.randint(0, 3, (E,))
    out = torch.zeros(B, E, F)
    L.local_masked_gather(x, idx, place, out, B, N, F, E, 1)
    keep = place == 1
    ref = torch.zeros(B, E, F)
    ref[:, keep] = x[:, idx[keep]]
    torch.testing.assert_close(out, ref)

    src = torch.randn(B, E, F)
    out2 = torch.zeros(B, R, F)
    L.local_masked_scatter(src, idx, place, out2, B, E, F, R, 2)
    ref2 = torch.zeros(B, R, F)
    for e in range(E):
        if place[e] == 2:
            ref2[:, idx[e] % R] += src[:, e]
    torch.testing.assert_close(out2, ref2)

    s = torch.randint(0, N, (E,))
    d = torch.randint(0, R, (E,))
    out3 = torch.zeros(B, R, F)
    L.local_masked_scatter_add_gather(x, s, d, out3, B, E, F, R)
    ref3 = torch.zeros(B, R, F)
    for e in range(E):
        ref3[:, d[e]] += x[:, s[e]]
    torch.testing.assert_close(out3, ref3)

    d_unique = torch.randperm(R)[:10]
    out4 = torch.zeros(B, R, F)
    L.local_masked_scatter_gather(x, s[:10], d_unique, out4, B, 10, F, R)
    ref4 = torch.zeros(B, R, F)
    ref4[:, d_unique] = x[:, s[:10]]
    torch.testing.assert_close(out4, ref4)


def test_rank_local_ops():
    from dgraph_amd.parallel import rank_local as RL

    x = torch.arange(40.0).reshape(1, 10, 4)
    idx = torch.tensor([[3, 1, 7, 7, 0]])
    rmap = torch.tensor([[0, 1, 0, 1, 0]])
    torch.testing.assert_close(RL.RankLocalMaskedGather(x, idx, rmap, 0), x[:, [3, 7, 0]])
    inv, uniq = RL.RankLocalReNumbering(torch.tensor([5, 2, 5, 9]))
    assert uniq.tolist() == [2, 5, 9] and inv.tolist() == [1, 0, 1, 2]
    inv, uniq, um = RL.RankLocalRenumberingWithMapping(torch.tensor([5, 2, 5, 9]),
                                                       torch.tensor([1, 0, 1, 2]))
    assert um.tolist() == [0, 1, 2]
    vals = torch.arange(8.0).reshape(1, 4, 2)
    agg, mapping = RL.LocalAggregateWithRemapping(vals, torch.tensor([5, 2, 5, 9]),
                                                  torch.tensor([1, 0, 1, 2]), 2, "cpu")
    torch.testing.assert_close(agg[0], torch.tensor([[2.0, 3.0], [4.0, 6.0], [6.0, 7.0]]))
    assert mapping.tolist() == [0, 1, 2]
    out = torch.zeros(1, 3, 2)
    RL.RankLocalMaskedScatter(vals, out, torch.tensor([[4, 2, 1, 0]]),
                              torch.tensor([[1, 1, 0, 1]]), 1)
    torch.testing.assert_close(out[0], torch.tensor([[6.0, 7.0], [0.0, 1.0], [2.0, 3.0]]))


# --------------------------------------------------------------------------- OGB wrapper
def _ogb_body(rank, world, tmp):
    from dgraph_amd import Communicator
    from dgraph_amd.data.ogbn import DistributedOGBWrapper

    comm = Communicator.init_process_group("gloo")
    ds = DistributedOGBWrapper("ogbn-arxiv", comm, dir_name=tmp, synthetic_scale=0.01)
    assert ds.synthetic and len(ds) == 1 and ds.num_classes == 40
    x, edges, rmaps, y = ds[0]
    g = ds.graph_obj
    n_loc = int(g.get_nodes_per_rank()[rank])
    assert x.shape == (n_loc, 128) and y.shape[0] == n_loc
    assert edges.shape[0] == 2 and rmaps.shape == edges.shape
    # every edge endpoint is owned by the rank its mapping names
    lo = torch.cat([torch.zeros(1, dtype=torch.long), g.get_nodes_per_rank().cumsum(0)])
    owner = torch.searchsorted(lo, edges.reshape(-1), right=True) - 1
    assert torch.equal(owner, rmaps.reshape(-1).long())
    comm.barrier()
    # second construction hits the cache file
    assert os.path.exists(os.path.join(tmp, f"ogbn-arxiv_graph_data_{world}.pt"))
    ds2 = DistributedOGBWrapper("ogbn-arxiv", comm, dir_name=tmp)
    assert torch.equal(ds2[0][0], x)


def test_ogb_wrapper_synthetic_two_ranks(tmp_path):
    run_ranks(_ogb_body, 2, str(tmp_path))


def test_ogb_wrapper_rejects_unknown(tmp_path):
    from dgraph_amd.data.ogbn import DistributedOGBWrapper

    with pytest.raises(AssertionError):
        DistributedOGBWrapper("ogbn-mag-not", None, dir_name=str(tmp_path))


# --------------------------------------------------------------------------- utils
def test_timing_report_cpu():
    from dgraph_amd.utils.timing import TimingReport

    TimingReport.init(None)
    for _ in range(3):
        TimingReport.start("step")
        sum(range(1000))
        TimingReport.stop("step")
    TimingReport.add_time("manual", 0.5)
    rep = TimingReport.report()
    assert rep["step"]["n"] == 3 and rep["manual"]["n"] == 1
    assert rep["step"]["mean_ms"] >= 0


def test_run_config_env_and_overrides():
    from dgraph_amd.utils.config import RunConfig, apply_overrides

    cfg = RunConfig.from_env({"DGRAPH_MODEL_HIDDEN": "64", "DGRAPH_KERNELS_SPMM_VARIANT": "1"})
    assert cfg.model.hidden == 64 and cfg.kernels.spmm_variant == 1
    apply_overrides(cfg, ["train.lr=0.5", "model.num_layers=4"])
    assert cfg.train.lr == 0.5 and cfg.model.num_layers == 4
    assert cfg.to_dict()["model"]["hidden"] == 64


def test_checkpoint_roundtrip(tmp_path):
    from dgraph_amd.models.sage import GraphSAGE
    from dgraph_amd.utils.checkpoint import load_checkpoint, plan_hash, save_checkpoint

    torch.manual_seed(0)
    m = GraphSAGE(16, 32, 5, num_layers=2)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    for p in m.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    h = plan_hash(torch.arange(10), extra="w1")
    path = str(tmp_path / "ck.pt")
    save_checkpoint(path, m, opt, epoch=7, plan_hash_value=h)
    m2 = GraphSAGE(16, 32, 5, num_layers=2)
    opt2 = torch.optim.Adam(m2.parameters(), lr=1e-3)
    st = load_checkpoint(path, m2, opt2, expected_plan_hash=h)
    assert st["epoch"] == 7 and not st["plan_stale"]
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)
    assert opt2.state_dict()["state"][0]["step"] == opt.state_dict()["state"][0]["step"]
    st = load_checkpoint(path, m2, expected_plan_hash="other")
    assert st["plan_stale"]
