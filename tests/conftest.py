"""Shared pytest configuration.

* ``gpu`` marker: tests that need a real MI355X (run with ``-m gpu`` on the GPU box);
  everything else runs on CPU.
* ``run_ranks(fn, world_size)``: spawn a CPU/gloo process group of ``world_size`` ranks
  on 127.0.0.1 and run ``fn(rank, world_size, *args)`` in each (the reference tested
  distribution only with torchrun on GPUs; this runs the same test bodies
  anywhere).
"""
from __future__ import annotations

import os
import socket
import sys
import traceback

import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and the native library")
    config.addinivalue_line("markers", "slow: long-running test")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world_size, port, fn, args, q, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world_size), LOCAL_RANK=str(rank))
    try:
        import torch.distributed as dist

        # W ranks share the container's CPUs: one intra-op pool each, sized to fit
        torch.set_num_threads(max(1, (os.cpu_count() or 8) // max(world_size, 1)))
        if backend in ("rccl", "gloo-multi-gpu"):
            # one rank per GPU (the reference's torchrun layout, tests/README.md:1-17):
            # rank r on cuda:r, RCCL over P2P/xGMI ("rccl") or gloo for the small
            # collectives with the data on distinct devices ("gloo-multi-gpu": the IPC heap)
            os.environ.update(DGRAPH_TEST_DEV=str(rank))
            torch.cuda.set_device(rank)
            if backend == "rccl":
                dist.init_process_group("nccl", rank=rank, world_size=world_size,
                                        device_id=torch.device("cuda", rank))
            else:
                dist.init_process_group("gloo", rank=rank, world_size=world_size)
        elif backend == "rccl-one-gpu":
            # real RCCL with every rank on GPU 0: RCCL refuses two ranks of one host on one
            # device ("Duplicate GPU"), so each rank names its own host and the ranks
            # connect over RCCL's socket transport on loopback (host-staged: a correctness
            # path for the RCCL code, not a bandwidth one)
            os.environ.update(NCCL_HOSTID=f"dgraph-test-rank{rank}", NCCL_SOCKET_IFNAME="lo",
                              LOCAL_RANK="0")
            torch.cuda.set_device(0)
            dist.init_process_group("nccl", rank=rank, world_size=world_size,
                                    device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world_size)
        torch.manual_seed(0)
        fn(rank, world_size, *args)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, None))
    except BaseException:
        q.put((rank, traceback.format_exc()))


def run_ranks(fn, world_size: int, *args, timeout: float = 240.0, backend: str = "gloo"):
    """Run ``fn(rank, world_size, *args)`` in ``world_size`` processes over a ``backend``
    process group (``"gloo"``; ``"rccl-one-gpu"``: RCCL with every rank on GPU 0; ``"rccl"``:
    RCCL with rank r on GPU r; ``"gloo-multi-gpu"``: gloo with rank r on GPU r); re-raise
    the first failure with its traceback. Test bodies take their device from
    :func:`rank_device`."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, fn, args, q, backend))
             for r in range(world_size)]
    for p in procs:
        p.start()
    errors = []
    for _ in procs:
        try:
            rank, err = q.get(timeout=timeout)
        except Exception:
            errors.append("timeout waiting for ranks")
            break
        if err:
            errors.append(f"rank {rank}:\n{err}")
    for p in procs:
        p.join(timeout=10)
        if p.is_alive():
            p.kill()
    if errors:
        raise AssertionError("\n".join(errors))


@pytest.fixture
def ranks():
    return run_ranks


def gpu_available() -> bool:
    return torch.cuda.is_available()


def rank_device() -> torch.device:
    """The GPU of this test rank: cuda:r under the one-rank-per-GPU backends, else cuda:0
    (ranks sharing the one-GPU box). Also makes it the current device."""
    dev = torch.device("cuda", int(os.environ.get("DGRAPH_TEST_DEV", "0")))
    torch.cuda.set_device(dev)
    return dev


def gpu_count() -> int:
    """Visible GPUs, without initialising the HIP runtime in the pytest process."""
    try:
        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def needs_gpus(n: int):
    """Skip (not fail) a test that maps its ranks to ``n`` distinct GPUs on a box with
    fewer (the 1-GPU box); an 8-GPU node runs it."""
    return pytest.mark.skipif(gpu_count() < n, reason=f"needs {n} GPUs (one rank per GPU), "
                                                      f"{gpu_count()} visible")
