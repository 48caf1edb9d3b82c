"""The exact bench.py training step as TWO PROCESSES on ONE GPU (W=2 across a real process
boundary, through the HIP kernels) against W=1 on the same GPU.

RCCL refuses two ranks per device, so the halo all-to-all-v runs on the one-sided
symmetric-heap transport (DGRAPH_A2A_IMPL=shmem: IPC-mapped peer heaps, puts at the
receivers' remote offsets — the reference's put contract, DGraph/distributed/Engine.py:
67-86); the small collectives (counts, gradient all-reduce) ride gloo. Rank 0 first runs the
W=1 job alone, then both ranks run the W=2 job; rank 0 compares losses, the first step's
all-reduced gradients, every parameter after 3 Adam steps and the validation/test hit
counts (reference: tests/test_NCCLCommPlan.py:85-124,242-359, replicated ground truth).

Covered: fp32 on the fused row-chunked executor (the headline path) in both graph
localities, at W = 2, 3 and 4; bf16 on the layer-stack path with halo recomputation off and on and the
gradient support prepared (the round-2 fused bf16 path).
"""
import argparse
import os
import types

import pytest
import torch
import torch.distributed as dist

from conftest import rank_device, run_ranks

pytestmark = pytest.mark.gpu


def _args(**kw):
    a = argparse.Namespace(shape="ogbn-papers100M", scale=2e-4, hidden=256, layers=3, lr=1e-2,
                           dtype="fp32", global_frac=0.05, window=256, seed=0,
                           no_overlap=False, rehearse_world=0, rehearse_rank=0,
                           halo_recompute="off", executor="auto", cuda_graph=False)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _run(rank, world, args, dtype, steps=3):
    import bench

    comm = types.SimpleNamespace(get_rank=lambda: rank, get_world_size=lambda: world,
                                 group=None)
    dev = rank_device()
    job = bench.Job(args, comm, dev, args.global_frac, dtype)
    if args.halo_recompute == "on" and world > 1:
        assert job.recompute, "halo recomputation was not enabled"
    if dtype == torch.float32:
        assert job.fused is not None, "fp32 must run on the fused executor"
    elif world > 1 and not job.recompute:
        assert job.graph.grad_support(job.train_idx) is not None, "grad support not prepared"
    grads = []
    orig = job.opt.step

    def capture(*a, **k):  # the gradients Adam consumes (all-reduced at W > 1)
        if not grads:
            grads.append([p.grad.detach().float().clone() for p in job.model.parameters()])
        return orig(*a, **k)

    job.opt.step = capture
    losses = []
    for _ in range(steps):
        loss = job.step(False).detach().float().clone()
        if world > 1:
            dist.all_reduce(loss)
        losses.append(float(loss))
    corr = job.correct.clone()
    if world > 1:
        dist.all_reduce(corr)
    out = {"losses": torch.tensor(losses, dtype=torch.float64), "grads": grads[0],
           "params": [p.detach().float().clone() for p in job.model.parameters()],
           "correct": corr.cpu(), "E_msg": job.E_msg, "halo": job.halo_total}
    job.free()
    torch.cuda.synchronize()
    return out


def _body(rank, world, kw, dt):
    rank_device()
    dtype = torch.float32 if dt == "fp32" else torch.bfloat16
    args = _args(dtype=dt, **{k: v for k, v in kw.items() if k != "stream_fill"})
    ref = _run(0, 1, args, dtype) if rank == 0 else None
    dist.barrier()
    got = _run(rank, world, args, dtype)
    from dgraph_amd.comm.alltoallv import close_shmem_heaps

    close_shmem_heaps()
    if rank != 0:
        return
    assert got["halo"] > 0, f"the W={world} partition has no halo: nothing crossed the boundary"
    assert ref["E_msg"] == got["E_msg"]
    if dt == "fp32":
        # the first step's loss to fp32 resolution; later losses after Adam steps: Adam moves
        # an entry whose (cancelling) gradient differs in rounding by a whole lr step, which
        # at a 512-wide hidden layer (2x the entries) shows in the loss at 3e-4 relative
        late = 1e-5 if args.hidden <= 256 else 2e-3
        torch.testing.assert_close(got["losses"][:1], ref["losses"][:1], atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(got["losses"][1:], ref["losses"][1:], atol=1e-5, rtol=late)
        # first-step gradients: fp32 rounding only (measured 1e-7 .. 7e-7 relative,
        # profiles/r03/multiproc_w2_vs_w1.log); the W=2 aggregation sums interior and halo
        # parts in another order
        # (streamed hidden layers run the self term as a separate GEMM during the pipeline
        # fill: one more fp32 rounding of every pre-activation than the W=1 dual GEMM, which
        # moves 512-wide hidden-layer gradients by 2-4e-5 relative through the few ReLU
        # gates it flips — 4e-7 with the fill off, scripts/debug/h512_w2_grads.py; an
        # aliasing error like ADVICE r4's is O(1))
        g_tol = 1e-4 if kw.get("stream_fill") else 1e-5
        for a, b in zip(got["grads"], ref["grads"]):
            rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
            assert rel < g_tol, f"W={world} gradient differs from W=1 by {rel:.2e} (relative)"
            assert float((a - b).abs().max()) <= 10 * g_tol * float(b.abs().max()) + 1e-9
        # after 3 Adam steps: Adam divides by sqrt(v), so a near-zero (cancelling) gradient
        # entry whose fp32 rounding differs moves by up to a whole lr step; everything else
        # must agree to fp32 resolution
        lr = args.lr
        for a, b in zip(got["params"], ref["params"]):
            d = (a - b).abs()
            assert float(d.max()) <= 3 * lr, float(d.max())   # never more than the 3 steps
            # on average: rounding (a 512-wide layer has 4x the weights near a ReLU tie or
            # a cancelling gradient, each moved by up to lr: 3.4e-3 lr on average measured)
            assert float(d.mean()) < (1e-3 if args.hidden <= 256 else 1e-2) * lr, \
                float(d.mean())
        assert torch.equal(got["correct"], ref["correct"])
    else:
        # bf16 storage: W=2 sums interior and halo parts in another order and rounds the
        # partial aggregate once more; compare at bf16 resolution
        torch.testing.assert_close(got["losses"], ref["losses"], atol=2e-3, rtol=2e-3)
        for a, b in zip(got["grads"], ref["grads"]):
            rel = float((a - b).norm() / b.norm().clamp_min(1e-12))
            assert rel < 3e-2, f"bf16 W=2 gradient differs from W=1 by {rel:.3e} (relative)"
        d = (got["correct"] - ref["correct"]).abs()
        assert int(d.max()) <= max(2, int(0.02 * int(ref["correct"].max()))), \
            (got["correct"], ref["correct"])


@pytest.mark.parametrize("dt,kw", [
    ("fp32", dict(global_frac=0.05)),
    ("fp32", dict(global_frac=1.0)),
    ("bf16", dict(global_frac=0.05, halo_recompute="off")),
    ("bf16", dict(global_frac=0.05, halo_recompute="on")),
    ("bf16", dict(global_frac=1.0, halo_recompute="on")),
], ids=["fp32-local", "fp32-structureless", "bf16-local", "bf16-local-recompute",
        "bf16-structureless-recompute"])
def test_bench_step_two_processes_one_gpu(monkeypatch, dt, kw):
    monkeypatch.setenv("DGRAPH_A2A_IMPL", "shmem")
    monkeypatch.setenv("DGRAPH_SYMHEAP_BYTES", str(1 << 30))
    run_ranks(_body, 2, kw, dt, timeout=240)


@pytest.mark.parametrize("world", [3, 4])
def test_bench_step_more_processes_one_gpu(monkeypatch, world):
    """W = 3 and 4 ranks (every rank exchanging with several peers at once) against W=1."""
    monkeypatch.setenv("DGRAPH_A2A_IMPL", "shmem")
    monkeypatch.setenv("DGRAPH_SYMHEAP_BYTES", str(1 << 30))
    run_ranks(_body, world, dict(global_frac=0.05), "fp32", timeout=110)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_alltoallv_shmem_processes(monkeypatch, world):
    """The shmem transport alone: random splits, two widths, two dtypes, repeated calls
    (slot reuse across calls must not leak into the next exchange)."""
    monkeypatch.setenv("DGRAPH_A2A_IMPL", "shmem")
    monkeypatch.setenv("DGRAPH_SYMHEAP_BYTES", str(64 << 20))
    run_ranks(_a2a_body, world, timeout=120)


def _a2a_body(rank, world, expect_mode=None):
    dev = rank_device()
    from dgraph_amd.comm.alltoallv import AllToAllV, close_shmem_heaps, shmem_heap

    g = torch.Generator().manual_seed(7)
    splits = torch.randint(0, 500, (world, world), generator=g)  # splits[src][dst]
    send_s = [int(v) for v in splits[rank]]
    recv_s = [int(splits[q][rank]) for q in range(world)]
    a2a = AllToAllV(send_s, recv_s)
    for it in range(3):
        for F, dt in ((64, torch.float32), (256, torch.bfloat16)):
            # row j of the block for peer p carries (src rank, dst rank, j, it)
            rows = []
            for p in range(world):
                j = torch.arange(send_s[p], dtype=torch.float32)
                v = (rank * 1000 + p * 100 + it) + j.unsqueeze(1) * 0.0 + \
                    torch.arange(F, dtype=torch.float32) * 0
                v[:, 0] = j
                rows.append(v)
            send = torch.cat(rows).to(dt).to(dev)
            out = a2a(send)
            torch.cuda.synchronize()
            off = 0
            for q in range(world):
                blk = out[off:off + recv_s[q]].float().cpu()
                exp = torch.full((recv_s[q], F), float(q * 1000 + rank * 100 + it))
                exp[:, 0] = torch.arange(recv_s[q], dtype=torch.float32)
                assert torch.equal(blk, exp.to(dt).float()), (rank, q, it, F)
                off += recv_s[q]
    heap = shmem_heap(None, dev)
    if expect_mode is not None:
        assert heap.device_completion == (expect_mode == "device"), expect_mode
        heap.check()
    used = heap._cursor
    close_shmem_heaps()
    assert used < (64 << 20)


@pytest.mark.parametrize("env", [{"DGRAPH_FUSED_BOUNDARY_STORE": "on"},
                                 {"DGRAPH_FUSED_HALO_STREAM": "on"},
                                 {"DGRAPH_FUSED_HALO_STREAM": "on",
                                  "DGRAPH_FUSED_STREAM_FILL": "0"}],
                         ids=["store", "stream", "stream-nofill"])
def test_bench_step_hidden512_two_processes(monkeypatch, env):
    """a 512-wide hidden layer at W=2 on the GPU kernels, through the two
    in-place aggregate-then-GEMM paths (boundary-row store, streamed halos), whose GEMM
    runs as column blocks with its aggregate operand aliasing the output."""
    monkeypatch.setenv("DGRAPH_A2A_IMPL", "shmem")
    monkeypatch.setenv("DGRAPH_SYMHEAP_BYTES", str(1 << 30))
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    # seed 1: with seed 0 one layer-1 pre-activation sits at a ReLU tie that the W=2
    # summation order flips (the hidden-layer gradients then differ by 2e-4 relative at
    # W=2 vs W=1 whatever the path; seeds 1 and 2: 2-4e-7, scripts/debug/h512_w2_grads.py)
    kw = dict(global_frac=0.05, hidden=512, seed=1)
    if "DGRAPH_FUSED_HALO_STREAM" in env and env.get("DGRAPH_FUSED_STREAM_FILL") != "0":
        # (the fill's one extra fp32 rounding: the looser gate; with the fill off the same
        # streamed in-place column-block path is held to the tight 1e-5 gate)
        kw["stream_fill"] = True
    run_ranks(_body, 2, kw, "fp32", timeout=240)


def _probe_body(rank, world):
    import bench

    dev = rank_device()
    args = _args(dtype="fp32", global_frac=0.05)
    comm = types.SimpleNamespace(get_rank=lambda: rank, get_world_size=lambda: world,
                                 group=None)
    job = bench.Job(args, comm, dev, args.global_frac, torch.float32)
    job.step(False)
    rec = bench.link_probe(job, width=64, iters=3)
    from dgraph_amd.comm.alltoallv import close_shmem_heaps

    job.free()
    torch.cuda.synchronize()
    close_shmem_heaps()
    assert rec["exchange_ms_max"] > 0, rec
    assert rec["largest_peer_message_GBps_min_over_ranks"] > 0, rec
    assert rec["transport"] == "shmem"


def test_bench_link_probe_two_processes(monkeypatch):
    """bench.py's W > 1 link probe (the achieved per-link rate of the job's own halo
    exchange, reported by the driver's multi-GPU runs) runs collectively and reports."""
    monkeypatch.setenv("DGRAPH_A2A_IMPL", "shmem")
    monkeypatch.setenv("DGRAPH_SYMHEAP_BYTES", str(1 << 30))
    run_ranks(_probe_body, 2, timeout=240)
