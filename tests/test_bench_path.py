"""The exact bench.py training step (``bench.Job``: partition build, DistGraph with the
overlapped halo exchange, full-graph GraphSAGE forward with validation/test logits from the
same forward, GradSync all-reduce, Adam) at W ranks reproduces W=1: same per-step losses,
same final weights and the same validation/test hit counts. Run on gloo at W = 2 and 8
(the 8-GPU node the round driver scales to), on the scaled papers100M shape, both graph
localities and the train-rows-only variant."""
import argparse
import types

import pytest
import torch

from conftest import run_ranks


def _args(**kw):
    a = argparse.Namespace(shape="ogbn-papers100M", scale=2e-5, hidden=128, layers=3, lr=1e-2,
                           dtype="fp32", global_frac=0.05, window=64, seed=0,
                           no_overlap=False, rehearse_world=0, rehearse_rank=0,
                           executor="stack")  # the layer-stack path (fused: below)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _run_job(rank, world, out, steps, global_frac, restrict, recompute="off",
             grad_support=True):
    import torch.distributed as dist

    import bench
    from dgraph_amd.parallel.dist_graph import DistGraph

    DistGraph.GRAD_SUPPORT = grad_support
    comm = types.SimpleNamespace(get_rank=lambda: rank, get_world_size=lambda: world,
                                 group=None)
    job = bench.Job(_args(global_frac=global_frac, halo_recompute=recompute), comm,
                    torch.device("cpu"), global_frac, torch.float32)
    if recompute == "on" and world > 1:
        assert job.recompute and job.graph.recompute is not None
    # the gradient support of the layer below the output layer is what the timed step
    # runs (bench.Job prepares it on every rank); a silently skipped build would leave the
    # dense transposed aggregation in its place and these tests would not see it
    sup = job.graph.grad_support(job.train_idx)
    assert (sup is not None) == grad_support, "grad support built / skipped unexpectedly"
    losses = []
    for _ in range(steps):
        loss = job.step(restrict).detach().clone()
        if world > 1:
            dist.all_reduce(loss)
        losses.append(float(loss))
    if recompute == "on" and world > 1:
        assert job.graph.recompute._cache, "the recompute path did not run"
    corr = job.correct.clone()
    if world > 1:
        dist.all_reduce(corr)
    DistGraph.GRAD_SUPPORT = True
    if rank == 0:
        torch.save({"losses": torch.tensor(losses, dtype=torch.float64),
                    "params": [p.detach().clone() for p in job.model.parameters()],
                    "correct": corr, "E_msg": job.E_msg, "n_train": job.n_train}, out)


@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("global_frac,restrict,chunked", [(0.05, False, False),
                                                          (1.0, False, False),
                                                          (0.05, True, False),
                                                          (1.0, False, True)])
def test_bench_step_matches_single_rank(tmp_path, monkeypatch, world, global_frac, restrict,
                                        chunked):
    """``chunked``: every halo exchange of width >= 128 is cut into 64-column chunks
    (DGRAPH_HALO_CHUNK_BYTES tiny), exercising the chunk pipeline of DistGraph."""
    if chunked:
        monkeypatch.setenv("DGRAPH_HALO_CHUNK_BYTES", "64")
    steps = 3
    _run_job(0, 1, tmp_path / "w1.pt", steps, global_frac, restrict)
    run_ranks(_run_job, world, str(tmp_path / "wn.pt"), steps, global_frac, restrict,
              timeout=600)
    a = torch.load(tmp_path / "w1.pt", weights_only=True)
    b = torch.load(tmp_path / "wn.pt", weights_only=True)
    assert a["E_msg"] == b["E_msg"] and a["n_train"] == b["n_train"]
    torch.testing.assert_close(a["losses"], b["losses"], atol=1e-5, rtol=1e-5)
    for p, q in zip(a["params"], b["params"]):
        torch.testing.assert_close(p, q, atol=1e-5, rtol=1e-4)
    if not restrict:
        # the last step's forward ran before its update: identical weights on entry
        assert torch.equal(a["correct"], b["correct"])


@pytest.mark.parametrize("world,global_frac,restrict", [(2, 0.05, False), (2, 1.0, False),
                                                        (4, 0.05, False), (4, 0.05, True),
                                                        (8, 0.05, False)])
def test_bench_step_halo_recompute_matches_single_rank(tmp_path, world, global_frac,
                                                       restrict):
    """Halo recomputation (parallel/halo_recompute.py): the first hidden layer computed
    for the halo rows on every rank, layer 2 exchanging nothing, reproduces W=1."""
    steps = 3
    _run_job(0, 1, tmp_path / "w1.pt", steps, global_frac, restrict)
    run_ranks(_run_job, world, str(tmp_path / "wn.pt"), steps, global_frac, restrict, "on",
              timeout=600)
    a = torch.load(tmp_path / "w1.pt", weights_only=True)
    b = torch.load(tmp_path / "wn.pt", weights_only=True)
    torch.testing.assert_close(a["losses"], b["losses"], atol=1e-5, rtol=1e-5)
    # the first layer's weight gradient sums the halo rows' share in another order (each
    # rank adds its own uses of a row): fp32 reassociation, amplified by Adam's 1/sqrt(v)
    for p, q in zip(a["params"], b["params"]):
        torch.testing.assert_close(p, q, atol=5e-5, rtol=1e-3)
    if not restrict:
        assert torch.equal(a["correct"], b["correct"])


@pytest.mark.parametrize("world,recompute", [(2, "off"), (4, "on")])
def test_bench_step_grad_support_on_off(tmp_path, world, recompute):
    """The gradient support (DistGraph.prepare_grad_support: the layer below the output
    layer aggregates transposed only from rows whose incoming gradient can be nonzero,
    including the halo sub-plan rows and, with recomputation, the extended halo rows) is
    exact: W ranks with the support built reproduce W ranks without it (the dense
    transposed aggregation) and W=1."""
    steps = 2
    run_ranks(_run_job, world, str(tmp_path / "on.pt"), steps, 0.05, False, recompute, True,
              timeout=600)
    run_ranks(_run_job, world, str(tmp_path / "off.pt"), steps, 0.05, False, recompute,
              False, timeout=600)
    a = torch.load(tmp_path / "on.pt", weights_only=True)
    b = torch.load(tmp_path / "off.pt", weights_only=True)
    torch.testing.assert_close(a["losses"], b["losses"], atol=1e-6, rtol=1e-6)
    for p, q in zip(a["params"], b["params"]):
        torch.testing.assert_close(p, q, atol=1e-5, rtol=1e-4)
    assert torch.equal(a["correct"], b["correct"])


def _run_job_fused(rank, world, out, steps, global_frac):
    import torch.distributed as dist

    import bench

    comm = types.SimpleNamespace(get_rank=lambda: rank, get_world_size=lambda: world,
                                 group=None)
    job = bench.Job(_args(global_frac=global_frac, hidden=256, halo_recompute="off",
                          executor="auto"), comm, torch.device("cpu"), global_frac,
                    torch.float32)
    assert job.fused is not None, "hidden 256 fp32 must take the fused executor"
    if world > 1:  # the forward exchanges overlap the next layer's interior aggregation
        assert job.fused.agg_full is not None
    grads = []
    orig = job.opt.step

    def capture(*a, **k):  # the (all-reduced) gradients of the first step
        if not grads:
            grads.append([p.grad.detach().clone() for p in job.model.parameters()])
        return orig(*a, **k)

    job.opt.step = capture
    losses = []
    for _ in range(steps):
        loss = job.step(False).detach().clone()
        if world > 1:
            dist.all_reduce(loss)
        losses.append(float(loss))
    corr = job.correct.clone()
    if world > 1:
        dist.all_reduce(corr)
    if rank == 0:
        torch.save({"losses": torch.tensor(losses, dtype=torch.float64), "grads": grads[0],
                    "params": [p.detach().clone() for p in job.model.parameters()],
                    "correct": corr, "E_msg": job.E_msg}, out)


@pytest.mark.parametrize("world,global_frac", [(2, 0.05), (2, 1.0), (8, 0.05)])
def test_bench_fused_step_matches_single_rank(tmp_path, world, global_frac):
    """The fp32 headline path (models/sage_fused.py through bench.Job) at W ranks
    reproduces W=1: per-step losses, weights after 3 Adam steps, validation/test hits."""
    steps = 3
    _run_job_fused(0, 1, tmp_path / "w1.pt", steps, global_frac)
    run_ranks(_run_job_fused, world, str(tmp_path / "wn.pt"), steps, global_frac,
              timeout=600)
    a = torch.load(tmp_path / "w1.pt", weights_only=True)
    b = torch.load(tmp_path / "wn.pt", weights_only=True)
    assert a["E_msg"] == b["E_msg"]
    torch.testing.assert_close(a["losses"], b["losses"], atol=1e-5, rtol=1e-5)
    for g, h in zip(a["grads"], b["grads"]):
        torch.testing.assert_close(g, h, atol=1e-7, rtol=1e-4)
    # each rank's weight-gradient partial sums its own rows before the all-reduce: fp32
    # reassociation, which Adam's 1/sqrt(v) amplifies for near-cancelling (near-zero)
    # gradient entries to a fraction of one lr step
    for p, q in zip(a["params"], b["params"]):
        torch.testing.assert_close(p, q, atol=2e-4, rtol=1e-3)
    assert torch.equal(a["correct"], b["correct"])
