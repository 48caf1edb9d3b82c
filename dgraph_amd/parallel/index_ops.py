"""Index-based distributed gather / scatter (API generation G1).

The reference's G1 NCCL path (``GatherFunction``/``ScatterFunction``,
_torch_func_impl.py:355-782) references undefined names and raises NameError whenever
data crosses ranks (D1). Here the intended semantics (tests/test_nccl_backend.py:294-405,
tests/test_mpi_backend.py:80-198, Engine.py:46-65) are implemented
by *lowering* the index arrays to an edge-centric plan on first use, caching it keyed by
the index tensors, and executing it with the G2 machinery (deterministic, no atomics).

Local row of a referenced vertex = ``index mod N_owner`` — identical to
``index - offset[owner]`` under the contiguous equal blocks the reference assumes
(_torch_func_impl.py:407,543).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..plan.nccl_plan import COO_to_NCCLCommPlan, NCCLGraphCommPlan
from .plan_ops import plan_gather, plan_scatter

_CACHE_SIZE = 64


def _comm_dev(group=None):
    from ..comm.groups import comm_device

    return comm_device(group)


def all_gather_counts(n: int, world_size: int, group=None) -> List[int]:
    if world_size == 1 or not dist.is_initialized():
        return [int(n)]
    t = torch.tensor([int(n)], dtype=torch.long, device=_comm_dev(group))
    parts = [torch.zeros_like(t) for _ in range(world_size)]
    dist.all_gather(parts, t, group=group)
    return [int(p.item()) for p in parts]


class G1PlanCache:
    """LRU cache of lowered G1 plans keyed by (index tensor identity, sizes)."""

    def __init__(self):
        self._d: "OrderedDict[tuple, NCCLGraphCommPlan]" = OrderedDict()

    @staticmethod
    def key(*tensors, extra=()) -> tuple:
        k = []
        for t in tensors:
            # identity + a position-weighted content checksum: a freed-and-reused
            # allocation with different indices must not hit a stale plan
            flat = t.reshape(-1).long()
            w = torch.arange(1, flat.numel() + 1, device=flat.device, dtype=torch.long)
            k += [t.data_ptr(), t.numel(), str(t.device), int((flat * w).sum())]
        return tuple(k) + tuple(extra)

    def get(self, key):
        p = self._d.get(key)
        if p is not None:
            self._d.move_to_end(key)
        return p

    def put(self, key, plan):
        self._d[key] = plan
        if len(self._d) > _CACHE_SIZE:
            self._d.popitem(last=False)

    def clear(self):
        self._d.clear()


def lower_local_form(
    indices: torch.Tensor,
    owners: torch.Tensor,
    num_local_rows: int,
    rank: int,
    world_size: int,
    group=None,
) -> NCCLGraphCommPlan:
    """Plan for this rank's edges referencing ``(owner, index)`` vertices."""
    sizes = all_gather_counts(num_local_rows, world_size, group)
    dev = indices.device
    sizes_t = torch.tensor(sizes, dtype=torch.long, device=dev)
    offset = torch.zeros(world_size + 1, dtype=torch.long, device=dev)
    offset[1:] = torch.cumsum(sizes_t, 0)
    idx = indices.reshape(-1).long().to(dev)
    own = owners.reshape(-1).long().to(dev)
    n_own = sizes_t[own].clamp(min=1)
    vgid = offset[own] + torch.remainder(idx, n_own)
    local_edges = torch.arange(idx.numel(), device=dev)
    return COO_to_NCCLCommPlan(rank, world_size, vgid, local_edges, offset, group)


def _as_batched(x: torch.Tensor) -> torch.Tensor:
    if x.dim() == 2:
        return x.unsqueeze(0)
    return x


def g1_gather_local(x, indices, owners, rank, world_size, cache: G1PlanCache, group=None):
    """MPI / NVSHMEM form: ``out[1, E_r, F]``, ``out[i] = X_owner(i)[indices[i] mod N]``."""
    x3 = _as_batched(x)
    key = G1PlanCache.key(indices, owners, extra=("g", x3.shape[1]))
    plan = cache.get(key)
    if plan is None:
        plan = lower_local_form(indices, owners, x3.shape[1], rank, world_size, group)
        cache.put(key, plan)
    return plan_gather(x3, plan, group)


def g1_scatter_local(x, indices, owners, num_output_rows, rank, world_size,
                     cache: G1PlanCache, group=None):
    """MPI / NVSHMEM form: ``out[1, N_r, F]``; owners receive the sum of contributions."""
    x3 = _as_batched(x)
    key = G1PlanCache.key(indices, owners, extra=("s", int(num_output_rows)))
    plan = cache.get(key)
    if plan is None:
        plan = lower_local_form(indices, owners, int(num_output_rows), rank, world_size, group)
        cache.put(key, plan)
    return plan_scatter(x3, plan, group)


def _select_local(indices: torch.Tensor, rank_mappings: torch.Tensor, rank: int
                  ) -> Tuple[torch.Tensor, torch.Tensor]:
    idx = indices.reshape(-1)
    rm = rank_mappings.reshape(2, -1) if rank_mappings.dim() != 2 else rank_mappings
    sel = torch.nonzero(rm[0].to(idx.device) == rank, as_tuple=True)[0]
    return idx[sel], rm[1].to(idx.device)[sel]


def g1_gather_global(x, indices, rank_mappings, rank, world_size, cache, group=None):
    """NCCL form: global ``indices[1,E]``, ``rank_mappings[2,E]`` = (edge placement,
    vertex owner). Returns ``[1, E_r, F]`` for the edges placed on this rank."""
    key = G1PlanCache.key(indices, rank_mappings, extra=("gg", x.shape[-2]))
    plan = cache.get(key)
    if plan is None:
        idx, own = _select_local(indices, rank_mappings, rank)
        plan = lower_local_form(idx, own, _as_batched(x).shape[1], rank, world_size, group)
        cache.put(key, plan)
    return plan_gather(_as_batched(x), plan, group)


def g1_scatter_global(x, indices, rank_mappings, output_size, rank, world_size, cache,
                      group=None):
    """NCCL form: ``x[1, E_r, F]`` holds this rank's edges (placement == rank, in order);
    returns ``[1, output_size, F]`` summed on the vertex owners."""
    key = G1PlanCache.key(indices, rank_mappings, extra=("gs", int(output_size)))
    plan = cache.get(key)
    if plan is None:
        idx, own = _select_local(indices, rank_mappings, rank)
        plan = lower_local_form(idx, own, int(output_size), rank, world_size, group)
        cache.put(key, plan)
    return plan_scatter(_as_batched(x), plan, group)


_LEGACY_CACHE = G1PlanCache()


class GatherFunction:
    """Reference-signature G1 gather (nccl/_torch_func_impl.py:355-579):
    ``GatherFunction.apply(local_send_tensor[1,N,F], indices[1,E], edge_rank_loc[E],
    edge_dest_ranks[E], rank, world_size)`` -> rows of the edges placed on ``rank``.
    Lowered once to a static plan (cached by content), then executed by the plan gather
    (autograd: the plan scatter), instead of re-deriving P2P send lists per call."""

    @staticmethod
    def apply(local_send_tensor, indices, edge_rank_loc, edge_dest_ranks, rank: int,
              world_size: int, group=None):
        rm = torch.stack([edge_rank_loc.reshape(-1), edge_dest_ranks.reshape(-1)])
        return g1_gather_global(local_send_tensor, indices, rm, rank, world_size,
                                _LEGACY_CACHE, group)


class ScatterFunction:
    """Reference-signature G1 scatter-sum (nccl/_torch_func_impl.py:582-782):
    ``ScatterFunction.apply(send_tensor[1,E_r,F], indices, edge_src_ranks, edge_dest_ranks,
    num_local_output_rows, rank, world_size)``."""

    @staticmethod
    def apply(send_tensor, indices, edge_src_ranks, edge_dest_ranks,
              num_local_output_rows: int, rank: int, world_size: int, group=None):
        rm = torch.stack([edge_src_ranks.reshape(-1), edge_dest_ranks.reshape(-1)])
        return g1_scatter_global(send_tensor, indices, rm, int(num_local_output_rows), rank,
                                 world_size, _LEGACY_CACHE, group)
