"""Process-group bootstrap and hybrid (graph-group x data-parallel) sub-communicators.

One process per GPU. On ROCm the torch backend named ``"nccl"`` *is* RCCL, so the GPU
path is RCCL over xGMI; CPU-only runs (the test-suite, config 1 of BASELINE.json) use
gloo with the identical code path. Replaces the ad-hoc ``dist.init_process_group``
calls of the reference (NCCLBackendEngine.py:49-64, MPIBackendEngine.py:310-317) and
implements the ``ranks_per_graph`` partition groups it only book-kept (P6, §2.5).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

_DEFAULT_TIMEOUT = datetime.timedelta(
    seconds=int(os.environ.get("DGRAPH_PG_TIMEOUT_S", "1800"))
)


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))


def default_device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", local_rank() % max(torch.cuda.device_count(), 1))
    return torch.device("cpu")


def ensure_process_group(backend: Optional[str] = None, **kwargs) -> bool:
    """Initialise the default process group if needed (env:// rendezvous, or a private
    single-rank store when no launcher variables are present). Returns True when this call
    created it (the caller then owns its teardown)."""
    if dist.is_initialized():
        return False
    if backend is None or backend == "auto":
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl" and not torch.cuda.is_available():
        backend = "gloo"
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    kw = dict(backend=backend, timeout=kwargs.pop("timeout", _DEFAULT_TIMEOUT))
    if backend == "nccl":
        if os.environ.get("DGRAPH_RCCL_SHARED_GPU") == "1":
            # several ranks on one device (a one-GPU test box): RCCL refuses two ranks of
            # one host on one device, so each rank names its own host and the ranks connect
            # over RCCL's socket transport on loopback — the RCCL code paths, host-staged
            os.environ["NCCL_HOSTID"] = f"dgraph-shared-gpu-rank{os.environ.get('RANK', '0')}"
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        dev = default_device()
        torch.cuda.set_device(dev)
        kw["device_id"] = dev
        if "pg_options" not in kwargs and os.environ.get("DGRAPH_PG_HIGH_PRIORITY", "1") == "1":
            # RCCL kernels on a high-priority stream: the halo exchange overlaps the
            # interior SpMM, and at equal priority the SpMM's waves fill every CU first
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            kw["pg_options"] = opts
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        dist.init_process_group(**kw, **kwargs)
    else:
        store = dist.HashStore()
        dist.init_process_group(store=store, rank=0, world_size=1, **kw, **kwargs)
    return True


@dataclass
class PartitionGroups:
    """``graph_group``: the ranks that jointly hold one vertex-partitioned graph;
    ``dp_group``: the ranks holding the same partition of different replicas."""

    ranks_per_graph: int
    partition_id: int
    partition_rank: int
    graph_group: Optional[dist.ProcessGroup]
    dp_group: Optional[dist.ProcessGroup]
    graph_ranks: List[int]
    dp_ranks: List[int]


def make_partition_groups(ranks_per_graph: int = -1) -> PartitionGroups:
    world = dist.get_world_size()
    rank = dist.get_rank()
    if ranks_per_graph in (-1, 0, None) or ranks_per_graph >= world:
        ranks_per_graph = world
    if world % ranks_per_graph != 0:
        raise ValueError(f"world size {world} not divisible by ranks_per_graph {ranks_per_graph}")
    pid, prank = divmod(rank, ranks_per_graph)
    graph_group = dp_group = None
    graph_ranks = list(range(pid * ranks_per_graph, (pid + 1) * ranks_per_graph))
    dp_ranks = list(range(prank, world, ranks_per_graph))
    if ranks_per_graph == world:
        graph_group = dist.group.WORLD
        if world > 1:
            # each rank is its own DP replica set of size 1: no DP communication needed
            dp_group = None
    else:
        # every rank must create every group, in the same order
        for p in range(world // ranks_per_graph):
            ranks = list(range(p * ranks_per_graph, (p + 1) * ranks_per_graph))
            g = dist.new_group(ranks)
            if p == pid:
                graph_group = g
        for r in range(ranks_per_graph):
            ranks = list(range(r, world, ranks_per_graph))
            g = dist.new_group(ranks)
            if r == prank:
                dp_group = g
    return PartitionGroups(ranks_per_graph, pid, prank, graph_group, dp_group,
                           graph_ranks, dp_ranks)


def comm_device(group: Optional[dist.ProcessGroup] = None) -> torch.device:
    """Device that tensors handed to collectives of ``group`` must live on."""
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")
