"""End-to-end trainer runs on CPU/gloo (synthetic data when ogb is absent): the OGB GCN
experiment at W=1 and W=2 gives the same loss trajectory and writes the reference's log
files."""
import os

import numpy as np
import pytest


def _ogb_gcn(rank, world, log_dir, out_path):
    import torch

    from dgraph_amd import Communicator
    from dgraph_amd.experiments import ogb_gcn
    from dgraph_amd.utils.timing import TimingReport

    torch.set_num_threads(2)
    tr, vl, va = ogb_gcn.main(backend="nccl", dataset="arxiv", epochs=4, lr=1e-2,
                              hidden_dims=32, log_dir=log_dir, synthetic_scale=0.01)
    if rank == 0:
        np.save(out_path, tr)
    TimingReport.reset()
    Communicator.instance().destroy()


@pytest.mark.parametrize("world", [1, 2])
def test_ogb_gcn_trainer(ranks, tmp_path, world):
    ranks(_ogb_gcn, world, str(tmp_path / "logs"), str(tmp_path / "loss.npy"))
    tr = np.load(tmp_path / "loss.npy")
    assert tr.shape == (1, 4) and np.isfinite(tr).all() and tr[0, -1] < tr[0, 0]
    for k in ("training_loss", "validation_accuracy", "test_results", "runtime_experiment"):
        assert os.path.exists(tmp_path / "logs" / f"arxiv_world{world}_run0_{k}.log")
    assert os.path.exists(tmp_path / "logs" / f"arxiv_timing_report_world{world}.json")
    ref = tmp_path.parent / f"gcn_loss_w{world}.npy"
    np.save(ref, tr)
    other = tmp_path.parent / f"gcn_loss_w{3 - world}.npy"
    if other.exists():  # W=1 and W=2 train the same model on the same data
        np.testing.assert_allclose(tr, np.load(other), rtol=1e-4, atol=1e-5)


def _lsc(rank, world, out_path, model="rgat"):
    import torch

    from dgraph_amd import Communicator
    from dgraph_amd.experiments import ogb_lsc

    torch.set_num_threads(2)
    trainer, final, accs = ogb_lsc.main(comm_type="nccl", num_papers=200, num_authors=300,
                                        num_institutions=12, num_features=8, num_classes=4,
                                        epochs=6, hidden_channels=16, heads=2, dropout=0.0,
                                        lr=1e-2, model=model)
    if rank == 0:
        np.save(out_path, np.array([h["loss"] for h in trainer.history] + list(accs)))
    Communicator.instance().destroy()


@pytest.mark.parametrize("model", ["rgat", "rgcn"])
def test_ogb_lsc_trainer_two_ranks(ranks, tmp_path, model):
    ranks(_lsc, 2, str(tmp_path / "lsc.npy"), model)
    r = np.load(tmp_path / "lsc.npy")
    losses, accs = r[:6], r[6:]
    assert np.isfinite(losses).all() and losses[-1] < losses[0]
    assert ((accs >= 0) & (accs <= 1)).all()


def _gc_train(rank, world, rpg, out_path, ckpt):
    import torch

    from dgraph_amd import Communicator
    from dgraph_amd.experiments import graphcast

    torch.set_num_threads(2)
    tr, last = graphcast.main(backend="nccl", procs_per_graph=rpg, iters=3, mesh_level=1,
                              grid="9x18", hidden_dim=8, processor_layers=1, channels=3,
                              checkpoint_dir=ckpt)
    if rank == 0:
        np.save(out_path, np.array([h["loss"] for h in tr.history]))
    Communicator.instance().destroy()


@pytest.mark.parametrize("world,rpg", [(1, -1), (2, -1), (2, 1)])
def test_graphcast_trainer(ranks, tmp_path, world, rpg):
    out = tmp_path / "gc.npy"
    ranks(_gc_train, world, rpg, str(out), str(tmp_path / "ck"))
    losses = np.load(out)
    assert losses.shape == (3,) and np.isfinite(losses).all()
    assert os.path.exists(tmp_path / "ck" / "model_3.pth")
    if rpg == -1:  # graph-parallel: identical trajectory to single process
        ref = tmp_path.parent / "gc_ref.npy"
        if world == 1:
            np.save(ref, losses)
        elif ref.exists():
            np.testing.assert_allclose(losses, np.load(ref), rtol=1e-4)


def _ogb_gcn_cli(rank, world, argv):
    import torch

    from dgraph_amd.experiments import ogb_gcn
    from dgraph_amd.utils.timing import TimingReport

    torch.set_num_threads(2)
    ogb_gcn.cli(argv)
    TimingReport.reset()


@pytest.mark.parametrize("world", [1, 2])
def test_ogb_gcn_resume_and_metrics(ranks, tmp_path, world):
    """--checkpoint_dir / --resume continue a run exactly (model, optimizer and RNG state
    restored): epochs 2-3 after a resume at epoch 2 repeat the uninterrupted run's losses;
    every epoch appends one JSONL metrics record (epoch_ms, edges_per_s, halo bytes per
    peer, peak HBM); --config overrides reach the RunConfig."""
    import json

    base = ["--backend", "nccl", "--dataset", "arxiv", "--lr", "1e-2", "--hidden_dims", "32",
            "--synthetic_scale", "0.01", "--config", "kernels.spmm_hub_cap=512"]
    full = str(tmp_path / "full")
    ranks(_ogb_gcn_cli, world, base + ["--epochs", "4", "--log_dir", full])
    part = str(tmp_path / "part")
    ck = str(tmp_path / "ck")
    ranks(_ogb_gcn_cli, world, base + ["--epochs", "2", "--log_dir", part,
                                       "--checkpoint_dir", ck])
    assert os.path.exists(os.path.join(ck, "checkpoint_latest.pt"))
    ranks(_ogb_gcn_cli, world, base + ["--epochs", "4", "--log_dir", part,
                                       "--resume", os.path.join(ck, "checkpoint_latest.pt")])

    def recs(d):
        with open(os.path.join(d, f"arxiv_world{world}_metrics.jsonl")) as f:
            return [json.loads(line) for line in f]

    a, b = recs(full), recs(part)
    assert [r["epoch"] for r in a] == [0, 1, 2, 3]
    assert [r["epoch"] for r in b] == [0, 1, 2, 3]  # 0-1 first run, 2-3 resumed
    for ra, rb in zip(a[2:], b[2:]):
        np.testing.assert_allclose(ra["loss"], rb["loss"], rtol=1e-5)
    for r in a:
        assert r["epoch_ms"] > 0 and r["edges_per_s"] > 0 and "peak_hbm_gb" in r
        if world > 1:
            assert r["halo_bytes_max_peer"] > 0 and r["halo_bytes_per_peer"]


def _gc_cli(rank, world, argv):
    import torch

    from dgraph_amd.experiments import graphcast
    from dgraph_amd.utils.timing import TimingReport

    torch.set_num_threads(2)
    graphcast.cli(argv)
    TimingReport.reset()


def test_graphcast_resume_bf16_master_weights(ranks, tmp_path):
    """GraphCast in bf16 keeps fp32 master weights (the checkpoint holds fp32 parameters)
    and resumes exactly: iterations 2-3 after a resume repeat the uninterrupted run."""
    import json

    import torch

    base = ["--backend", "nccl", "--mesh_level", "1", "--grid", "9x18", "--hidden_dim", "8",
            "--processor_layers", "1", "--channels", "3", "--dtype", "bf16"]
    ranks(_gc_cli, 1, base + ["--iters", "4", "--log_dir", str(tmp_path / "a")])
    ck = str(tmp_path / "ck")
    ranks(_gc_cli, 1, base + ["--iters", "2", "--log_dir", str(tmp_path / "b"),
                              "--checkpoint_dir", ck])
    state = torch.load(os.path.join(ck, "checkpoint_latest.pt"), weights_only=True)
    assert all(v.dtype == torch.float32 for k, v in state["model"].items()
               if v.is_floating_point()), "masters must be saved in fp32"
    ranks(_gc_cli, 1, base + ["--iters", "4", "--log_dir", str(tmp_path / "b"),
                              "--resume", os.path.join(ck, "checkpoint_latest.pt")])

    def recs(d):
        name = [f for f in os.listdir(d) if f.endswith("_metrics.jsonl")][0]
        with open(os.path.join(d, name)) as f:
            return [json.loads(line) for line in f]

    a, b = recs(tmp_path / "a"), recs(tmp_path / "b")
    assert [r["epoch"] for r in b] == [0, 1, 2, 3]
    np.testing.assert_allclose([r["loss"] for r in a[2:]], [r["loss"] for r in b[2:]],
                               rtol=1e-5)
