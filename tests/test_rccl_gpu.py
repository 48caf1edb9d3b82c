"""Real RCCL at W > 1 on a ONE-GPU box: every rank on GPU 0, each naming its own host
(NCCL_HOSTID) so RCCL accepts the pair and connects it over its socket transport on loopback
(conftest.run_ranks(backend="rccl-one-gpu")). Slow and host-staged, but the RCCL code paths
are the ones the multi-GPU node runs:

* the torch ProcessGroupNCCL all-to-all-v (DGRAPH_A2A_IMPL=torch, the default transport),
* the native grouped send/recv executor (DGRAPH_A2A_IMPL=native, comm/rccl_exec.py) on its
  own RCCL communicator, synchronous and asynchronous on its high-priority stream,
* the exact bench.py fp32 training step at W=2 over either against W=1 (gradient
  all-reduce over RCCL too), and bench.py's link probe with the executor A/B.

Reference: DGraph/distributed/nccl/alltoallv_impl.py:110-123 (per-peer NCCL P2P),
tests/test_NCCLCommPlan.py (W>1 against replicated ground truth).
"""
import pytest
import torch

from conftest import rank_device, run_ranks

pytestmark = pytest.mark.gpu


def _a2a_body(rank, world):
    import torch.distributed as dist

    from dgraph_amd.comm import alltoallv as A

    assert dist.get_backend() == "nccl"
    g = torch.Generator().manual_seed(11)
    splits = torch.randint(0, 400, (world, world), generator=g)
    splits[0, 1] = 0  # a zero-size peer (skipped by the executor)
    send_s = [int(v) for v in splits[rank]]
    recv_s = [int(splits[q][rank]) for q in range(world)]
    a2a = A.AllToAllV(send_s, recv_s)
    dev = rank_device()
    for it in range(2):
        for F, dt in ((64, torch.float32), (200, torch.bfloat16)):
            send = torch.cat([torch.full((n, F), float(rank * 1000 + p * 100 + it))
                              for p, n in enumerate(send_s)]).to(dt).to(dev)
            send[:, 0] = torch.arange(send.shape[0], dtype=torch.float32).to(dt)
            exp = []
            for q in range(world):
                e = torch.full((recv_s[q], F), float(q * 1000 + rank * 100 + it))
                e[:, 0] = sum(int(splits[q][p]) for p in range(rank)) + \
                    torch.arange(recv_s[q], dtype=torch.float32)
                exp.append(e)
            exp = torch.cat(exp).to(dt)
            out = a2a(send)
            torch.cuda.synchronize()
            assert torch.equal(out.cpu(), exp), (rank, it, F, "sync")
            # asynchronous from a side stream, consumed on the compute stream after wait()
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                out2, work = a2a(send, async_op=True)
            work.wait()
            got = (out2.float() * 1.0).cpu()
            torch.cuda.synchronize()
            assert torch.equal(got, exp.float()), (rank, it, F, "async")
    from dgraph_amd.comm.rccl_exec import RCCLExecutor

    RCCLExecutor.close_all()


@pytest.mark.parametrize("impl", ["torch", "native"])
def test_alltoallv_rccl_two_ranks(monkeypatch, impl):
    monkeypatch.setenv("DGRAPH_A2A_IMPL", impl)
    run_ranks(_a2a_body, 2, timeout=180, backend="rccl-one-gpu")


def _step_body(rank, world, impl):
    import test_multiproc_gpu as T

    from dgraph_amd.comm.rccl_exec import RCCLExecutor

    T._body(rank, world, dict(global_frac=0.05), "fp32")
    RCCLExecutor.close_all()


@pytest.mark.parametrize("impl", ["torch", "native"])
def test_bench_step_rccl_two_ranks(monkeypatch, impl):
    """The fused fp32 bench step at W=2 with its halo exchanges and gradient all-reduce on
    RCCL, against W=1 (same tolerances as the shmem-transport test)."""
    monkeypatch.setenv("DGRAPH_A2A_IMPL", impl)
    run_ranks(_step_body, 2, impl, timeout=240, backend="rccl-one-gpu")


def _probe_body(rank, world):
    import types

    import bench
    import test_multiproc_gpu as T

    from dgraph_amd.comm.rccl_exec import RCCLExecutor

    args = T._args(dtype="fp32", global_frac=0.05)
    comm = types.SimpleNamespace(get_rank=lambda: rank, get_world_size=lambda: world,
                                 group=None)
    job = bench.Job(args, comm, rank_device(), args.global_frac, torch.float32)
    job.step(False)
    rec = bench.link_probe(job, width=64, iters=2)
    job.free()
    torch.cuda.synchronize()
    RCCLExecutor.close_all()
    assert rec["transport"] == "torch", rec
    assert rec["exchange_ms_max"] > 0, rec
    nat = rec["native_executor"]
    assert nat.get("bitwise_equal_to_torch") is True, rec
    assert nat["exchange_ms_max"] > 0, rec


def test_bench_link_probe_native_ab_rccl(monkeypatch):
    """bench.py's W > 1 link probe on RCCL: the torch transport timed, then the native
    executor on the same send rows, bitwise equal to it, timed."""
    monkeypatch.setenv("DGRAPH_A2A_IMPL", "torch")
    run_ranks(_probe_body, 2, timeout=240, backend="rccl-one-gpu")


def _bench(args, env_extra, timeout=400):
    import json
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, **env_extra)
    p = subprocess.run([sys.executable, "-u", os.path.join(repo, "bench.py")] + args,
                       cwd=repo, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_cli_two_ranks_rccl_shared_gpu():
    """The driver's multi-GPU path end to end on one GPU: ``bench.py --gpus 2`` launches
    its ranks with torch.distributed.run, both on GPU 0 over real RCCL
    (DGRAPH_RCCL_SHARED_GPU=1: per-rank NCCL_HOSTID, socket transport); ONE JSON line, the
    RCCL world of 2, the link probe with the native-executor A/B bitwise equal, and the
    same loss as the W=1 run of the same (reduced-scale) graph."""
    common = ["--scale", "0.02", "--steps", "2", "--warmup", "1", "--no-extra"]
    w1 = _bench(["--gpus", "1"] + common, {})
    w2 = _bench(["--gpus", "2"] + common, {"DGRAPH_RCCL_SHARED_GPU": "1"})
    assert w2["n_gpus"] == 2 and w2["config"]["rccl_world_size"] == 2
    assert w2["config"]["process_group_backend"] == "nccl"
    assert w2["xgmi_probe"]["native_executor"]["bitwise_equal_to_torch"] is True
    assert abs(w2["final_loss"] - w1["final_loss"]) <= 1e-4 * abs(w1["final_loss"])
    assert w2["val_acc"] == w1["val_acc"] and w2["test_acc"] == w1["test_acc"]
