"""Backend ``"rocshmem"`` (alias ``"nvshmem"``): one-sided symmetric-heap engine.

Counterpart of the reference's ``NVSHMEMBackendEngine`` + ``torch_nvshmem_p2p``
(nvshmem/NVSHMEMBackendEngine.py:163-315, csrc/torch_nvshmem_p2p.cu:32-376).
rocSHMEM is not installed in this image, so the symmetric heap is the native HIP-IPC
heap in ``csrc/comm/symheap.hip`` (:class:`dgraph_amd.comm.symheap.SymmetricHeap`):
every rank maps every peer's heap over xGMI, remote rows are read with wave64 16-byte
peer loads (the K15 remote get) and written with peer stores at ``remote_offsets`` (put),
one-sided scatter puts pre-summed rows into per-source slots of the owner's heap (summed
there in a fixed order), and completion is stream-ordered (device-side signal / wait). Sizes are agreed as the max over ranks
(fixing the reference's mismatched collective ``nvshmem_malloc`` sizes, D4).

When the heap cannot be used (host tensors, a single process spanning several nodes, or
``DGRAPH_SHMEM_TRANSPORT=two_sided``) the engine executes the same one-sided semantics
through the two-sided plan path, so results are identical on every transport.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .alltoallv import AllToAllV, offsets_to_splits
from .base import BackendEngine
from .groups import ensure_process_group, make_partition_groups


class ROCSHMEMBackendEngine(BackendEngine):
    _is_initialized = False
    _ranks_per_graph = -1
    _partition_num = 0

    def __init__(self, ranks_per_graph: int = -1, **kwargs):
        from ..parallel.index_ops import G1PlanCache

        self._g1_cache = G1PlanCache()
        self._heap = None
        self.init_process_group(ranks_per_graph, **kwargs)

    def init_process_group(self, ranks_per_graph: int = -1, **kwargs):
        pgb = kwargs.pop("pg_backend", None)
        self._owns_pg = ensure_process_group(pgb or kwargs.pop("backend", None), **kwargs)
        self._groups = make_partition_groups(ranks_per_graph)
        ROCSHMEMBackendEngine._ranks_per_graph = self._groups.ranks_per_graph
        ROCSHMEMBackendEngine._partition_num = self._groups.partition_id
        ROCSHMEMBackendEngine._is_initialized = True
        self.transport = os.environ.get("DGRAPH_SHMEM_TRANSPORT", "auto")

    @property
    def group(self):
        g = self._groups.graph_group
        return None if g is dist.group.WORLD else g

    def heap(self):
        """Lazily created device symmetric heap (None when unavailable)."""
        if self._heap is None and self.transport != "two_sided" and torch.cuda.is_available():
            from .symheap import SymmetricHeap

            try:
                self._heap = SymmetricHeap.create(self.group)
            except Exception as e:  # pragma: no cover - depends on IPC support
                if self.transport == "ipc":
                    raise
                self.transport = "two_sided"
                self._heap_error = e
        return self._heap

    def get_rank(self) -> int:
        return self._groups.partition_rank

    def get_world_size(self) -> int:
        return self._groups.ranks_per_graph

    def get_local_rank_slice(self, tensor: torch.Tensor, dim: int = -1) -> torch.Tensor:
        W, r = self.get_world_size(), self.get_rank()
        size = tensor.shape[dim] // W
        return tensor.narrow(dim, r * size, size)

    def allocate_buffer(self, size, dtype, device):
        h = self.heap() if torch.device(device).type == "cuda" else None
        if h is not None:
            return h.alloc_tensor(size, dtype)
        return torch.empty(size, dtype=dtype, device=device)

    def put(self, send_buffer, recv_buffer, send_offsets, recv_offsets, remote_offsets=None):
        h = self.heap() if send_buffer.is_cuda else None
        if h is not None and remote_offsets is not None and h.owns(recv_buffer):
            h.put_rows(send_buffer, recv_buffer, offsets_to_splits(send_offsets),
                       remote_offsets)
            return
        AllToAllV(offsets_to_splits(send_offsets), offsets_to_splits(recv_offsets),
                  self.group)(send_buffer, out=recv_buffer)

    def gather(self, x, indices, rank_mappings, *args, **kwargs):
        from ..parallel import index_ops

        x3 = x if x.dim() == 3 else x.unsqueeze(0)
        assert x3.shape[0] == 1, "Batch size must be 1"
        h = self.heap() if x3.is_cuda else None
        if h is not None:
            return h.remote_gather(x3[0], indices.reshape(-1), rank_mappings.reshape(-1)).unsqueeze(0)
        return index_ops.g1_gather_local(x3, indices, rank_mappings, self.get_rank(),
                                         self.get_world_size(), self._g1_cache, self.group)

    def scatter(self, x, indices, rank_mappings, num_output_rows, *args, **kwargs):
        from ..parallel import index_ops

        x3 = x if x.dim() == 3 else x.unsqueeze(0)
        h = self.heap() if x3.is_cuda else None
        if h is not None:
            # one-sided: pre-summed rows put into the owners' slots, fixed-order add there
            return h.scatter_add(x3[0], indices.reshape(-1), rank_mappings.reshape(-1),
                                 int(num_output_rows)).unsqueeze(0)
        return index_ops.g1_scatter_local(x, indices, rank_mappings, num_output_rows,
                                          self.get_rank(), self.get_world_size(),
                                          self._g1_cache, self.group)

    def get_max(self, val: int) -> int:
        t = torch.tensor([int(val)], dtype=torch.long,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def barrier(self) -> None:
        h = self._heap
        if h is not None:
            h.barrier()
        dist.barrier()

    def finalize(self) -> None:
        if self._heap is not None:
            self._heap.close()
            self._heap = None
        ROCSHMEMBackendEngine._is_initialized = False

    def destroy(self) -> None:
        self.finalize()
        self._g1_cache.clear()
        if getattr(self, "_owns_pg", False) and dist.is_initialized():
            self._owns_pg = False
            dist.destroy_process_group()


# API-compatibility alias (reference backend name "nvshmem")
NVSHMEMBackendEngine = ROCSHMEMBackendEngine
