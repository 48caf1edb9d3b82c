"""The single user entry point: ``Communicator.init_process_group(backend)``.

Same API as the reference's facade (DGraph/Communicator.py:24-141): process-wide
singleton, ``get_rank/get_world_size/get_local_rank_slice/get_local_tensor/alloc_buffer/
scatter/gather/put/barrier/destroy``. Backends: ``"nccl"`` (RCCL over xGMI; gloo on CPU),
``"mpi"`` (host-capable), ``"rocshmem"``/``"nvshmem"`` (one-sided symmetric heap).
Unlike the reference, constructor kwargs (``ranks_per_graph``) reach every engine, and
the plan caches / timers the apps need are public (``engine``, ``group``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .base import CommunicatorBase

SUPPORTED_BACKENDS = ["nccl", "mpi", "nvshmem", "rocshmem", "gloo"]


def _make_engine(backend: str, **kwargs):
    if backend in ("nccl", "gloo"):
        from .nccl_engine import NCCLBackendEngine

        if backend == "gloo":
            kwargs.setdefault("backend", "gloo")
        return NCCLBackendEngine(**kwargs)
    if backend == "mpi":
        from .mpi_engine import MPIBackendEngine

        return MPIBackendEngine(**kwargs)
    if backend in ("nvshmem", "rocshmem"):
        from .shmem_engine import ROCSHMEMBackendEngine

        return ROCSHMEMBackendEngine(**kwargs)
    raise NotImplementedError(f"Backend {backend} not implemented")


class Communicator(CommunicatorBase):
    _is_initialized = False
    _instance: Optional["Communicator"] = None

    def __init__(self, backend: str, **kwargs) -> None:
        super().__init__()
        if backend not in SUPPORTED_BACKENDS:
            raise AssertionError(
                f"Backend {backend} not supported. Supported backends: {SUPPORTED_BACKENDS}")
        self.backend = backend
        self.kwargs = kwargs
        self._engine = _make_engine(backend, **kwargs)
        Communicator._is_initialized = True
        Communicator._instance = self

    @staticmethod
    def init_process_group(backend: str, **kwargs) -> "Communicator":
        if Communicator._is_initialized:
            raise RuntimeError("Communicator already initialized")
        return Communicator(backend, **kwargs)

    @staticmethod
    def instance() -> "Communicator":
        if Communicator._instance is None or not Communicator._is_initialized:
            raise RuntimeError("Communicator not initialized")
        return Communicator._instance

    # -- engine access (public; the reference apps reached into a private attribute) --
    @property
    def engine(self):
        return self._engine

    @property
    def group(self):
        return getattr(self._engine, "group", None)

    @property
    def partition(self):
        """:class:`~dgraph_amd.comm.groups.PartitionGroups` (graph group x replica group),
        or None for engines without ``ranks_per_graph`` support."""
        return getattr(self._engine, "_groups", None)

    def partition_rank(self) -> int:
        """Rank inside this process's graph group (== get_rank() without replicas)."""
        p = self.partition
        return p.partition_rank if p is not None else self.get_rank()

    def partition_size(self) -> int:
        p = self.partition
        return p.ranks_per_graph if p is not None else self.get_world_size()

    def _check(self):
        assert Communicator._is_initialized, "Communicator not initialized"

    def get_rank(self) -> int:
        self._check()
        return self._engine.get_rank()

    def get_world_size(self) -> int:
        self._check()
        return self._engine.get_world_size()

    def get_local_rank_slice(self, tensor: torch.Tensor, dim: int = -1) -> torch.Tensor:
        self._check()
        return self._engine.get_local_rank_slice(tensor, dim)

    def get_local_tensor(self, tensor: torch.Tensor, placement_tensor: torch.Tensor,
                         dim: int = -1) -> torch.Tensor:
        """Rows of ``tensor`` along ``dim`` whose placement equals this rank."""
        self._check()
        sel = torch.nonzero(placement_tensor.reshape(-1) == self.get_rank(), as_tuple=True)[0]
        return tensor.index_select(dim, sel.to(tensor.device))

    def alloc_buffer(self, size: Tuple[int, ...], dtype: torch.dtype,
                     device: torch.device) -> torch.Tensor:
        return self._engine.allocate_buffer(size, dtype, device)

    def scatter(self, *args, **kwargs) -> torch.Tensor:
        self._check()
        return self._engine.scatter(*args, **kwargs)

    def gather(self, *args, **kwargs) -> torch.Tensor:
        self._check()
        return self._engine.gather(*args, **kwargs)

    def put(self, send_buffer, recv_buffer, send_offsets, recv_offsets,
            remote_offsets=None) -> None:
        self._check()
        return self._engine.put(send_buffer, recv_buffer, send_offsets, recv_offsets,
                                remote_offsets=remote_offsets)

    def barrier(self) -> None:
        self._check()
        self._engine.barrier()

    def destroy(self) -> None:
        self._check()
        try:
            self._engine.destroy()
        finally:
            Communicator._is_initialized = False
            Communicator._instance = None
