"""Backend ``"nccl"``: RCCL over xGMI (two-sided).

Counterpart of the reference's ``NCCLBackendEngine`` (nccl/NCCLBackendEngine.py:35-318).
On ROCm the torch process-group backend named ``"nccl"`` is RCCL; the same engine runs
on a gloo group when no GPU is present (tests, CPU configs). Provides:

* ``put``: host-split all-to-all-v (splits cached per offsets tensor, no per-call sync);
* ``gather``/``scatter`` with ``comm_plan=`` (G2) or ``(indices, rank_mappings)`` (G1,
  lowered to cached plans — fixing the reference's broken legacy path, D1);
* ``ranks_per_graph`` hybrid partitioning: graph-group sub-communicator (all graph
  collectives run in it, ranks are partition-local) x replica groups (P6).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .alltoallv import AllToAllV, offsets_to_splits
from .base import BackendEngine
from .groups import PartitionGroups, ensure_process_group, make_partition_groups

TIMINGS: Dict[str, list] = {}


class NCCLBackendEngine(BackendEngine):
    _is_initialized = False
    _groups: Optional[PartitionGroups] = None

    def __init__(self, ranks_per_graph: int = -1, *args, **kwargs):
        self._split_cache: Dict[tuple, Tuple[List[int], List[int]]] = {}
        from ..parallel.index_ops import G1PlanCache

        self._g1_cache = G1PlanCache()
        if not NCCLBackendEngine._is_initialized:
            self.init_process_group(ranks_per_graph, *args, **kwargs)

    # ------------------------------------------------------------------ setup
    def init_process_group(self, ranks_per_graph: int = -1, *args, **kwargs):
        backend = kwargs.pop("pg_backend", None) or kwargs.pop("backend", None)
        NCCLBackendEngine._owns_pg = ensure_process_group(backend or "nccl", **kwargs)
        NCCLBackendEngine._groups = make_partition_groups(ranks_per_graph)
        NCCLBackendEngine._is_initialized = True

    @property
    def group(self) -> Optional[dist.ProcessGroup]:
        g = NCCLBackendEngine._groups
        return None if g is None or g.graph_group is dist.group.WORLD else g.graph_group

    @staticmethod
    def get_rank() -> int:
        return dist.get_rank()

    @staticmethod
    def get_world_size() -> int:
        return dist.get_world_size()

    @staticmethod
    def get_local_rank() -> int:
        return NCCLBackendEngine._groups.partition_rank

    @staticmethod
    def get_partition_size() -> int:
        return NCCLBackendEngine._groups.ranks_per_graph

    @staticmethod
    def get_partition_id() -> int:
        return NCCLBackendEngine._groups.partition_id

    def get_local_rank_slice(self, tensor: torch.Tensor, dim: int = -1) -> torch.Tensor:
        """Equal contiguous slice of dim 1 for this partition rank (reference semantics:
        the NCCL engine ignores ``dim``, NCCLBackendEngine.py:86-94)."""
        n = self.get_partition_size()
        r = self.get_local_rank()
        size = tensor.shape[1] // n
        return tensor[:, r * size:(r + 1) * size]

    # ------------------------------------------------------------------ data plane
    def _splits(self, send_offsets, recv_offsets) -> Tuple[List[int], List[int]]:
        def k(t):
            if isinstance(t, torch.Tensor):
                return (t.data_ptr(), t.numel(), t._version, str(t.device))
            return tuple(t)

        key = (k(send_offsets), k(recv_offsets))
        v = self._split_cache.get(key)
        if v is None:
            v = (offsets_to_splits(send_offsets), offsets_to_splits(recv_offsets))
            if len(self._split_cache) > 256:
                self._split_cache.clear()
            self._split_cache[key] = v
        return v

    def put(self, send_buffer, recv_buffer, send_offsets, recv_offsets,
            remote_offsets=None) -> None:
        _ = remote_offsets  # two-sided
        ss, rs = self._splits(send_offsets, recv_offsets)
        AllToAllV(ss, rs, self.group)(send_buffer, out=recv_buffer)

    def alltoallv(self, send_splits, recv_splits) -> AllToAllV:
        return AllToAllV(send_splits, recv_splits, self.group)

    def gather(self, x: torch.Tensor, indices: Optional[torch.Tensor] = None,
               rank_mappings: Optional[torch.Tensor] = None, *, comm_plan=None, **kw):
        from ..parallel import index_ops
        from ..parallel.plan_ops import plan_gather

        if comm_plan is not None:
            return plan_gather(x, comm_plan, self.group)
        if kw.get("cache") is not None:  # NCCLGatherCache from the G1 cache generators
            return plan_gather(x, kw["cache"].plan, self.group)
        if indices is None or rank_mappings is None:
            raise ValueError("gather needs comm_plan= or (indices, rank_mappings)")
        return index_ops.g1_gather_global(x, indices, rank_mappings, self.get_local_rank(),
                                          self.get_partition_size(), self._g1_cache, self.group)

    def scatter(self, x: torch.Tensor, indices: Optional[torch.Tensor] = None,
                rank_mappings: Optional[torch.Tensor] = None, output_size: Optional[int] = None,
                *, comm_plan=None, **kw):
        from ..parallel import index_ops
        from ..parallel.plan_ops import plan_scatter

        if comm_plan is not None:
            return plan_scatter(x, comm_plan, self.group)
        if kw.get("cache") is not None:  # NCCLScatterCache
            return plan_scatter(x, kw["cache"].plan, self.group)
        if indices is None or rank_mappings is None or output_size is None:
            raise ValueError("scatter needs comm_plan= or (indices, rank_mappings, output_size)")
        return index_ops.g1_scatter_global(x, indices, rank_mappings, output_size,
                                           self.get_local_rank(), self.get_partition_size(),
                                           self._g1_cache, self.group)

    # ------------------------------------------------------------------ control
    def barrier(self) -> None:
        if not NCCLBackendEngine._is_initialized:
            raise RuntimeError("NCCLBackendEngine is not initialized, cannot call barrier")
        dist.barrier()

    def finalize(self) -> None:
        if NCCLBackendEngine._is_initialized:
            dist.barrier()

    def destroy(self) -> None:
        NCCLBackendEngine._is_initialized = False
        NCCLBackendEngine._groups = None
        self._g1_cache.clear()
        if getattr(NCCLBackendEngine, "_owns_pg", False) and dist.is_initialized():
            # the engine created the process group: tear it down (RCCL communicators
            # included) instead of leaving it to interpreter exit
            NCCLBackendEngine._owns_pg = False
            dist.destroy_process_group()
