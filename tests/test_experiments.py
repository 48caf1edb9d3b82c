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
