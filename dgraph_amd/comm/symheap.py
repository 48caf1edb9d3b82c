"""Symmetric device heap over HIP IPC — the one-sided transport of the ``rocshmem`` /
``nvshmem`` backend (replaces NVSHMEM: DGraph/distributed/csrc/torch_nvshmem_p2p.cu:32-376,
nvshmem_comm_kernels.cuh:60-170).

Every rank of the group ``hipMalloc``'s one heap of the same size (the max of the requested
sizes — the reference's collective ``nvshmem_malloc`` was called with per-rank sizes, D4),
publishes its IPC handle, and maps every peer heap. Tensors carved from the heap with
:meth:`SymmetricHeap.alloc_tensor` live at the same offset on every rank (allocation is a
collective bump allocator: all ranks allocate in the same order), so a peer's copy of a
symmetric tensor is ``peer_base[p] + offset``. Native kernels (csrc/comm/symheap.hip) then

* read remote rows directly over xGMI (:meth:`remote_gather`, the K15 ``dist_get``), and
* write rows into peers' receive buffers at ``remote_offsets`` (:meth:`put_rows`).

Completion is host-ordered: drain the current stream, then a process-group barrier
(:meth:`barrier`). Accumulating remote puts (the reference's CAS-loop ``dist_put``) go through
the two-sided scatter path instead of remote atomics.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import _native

_ALIGN = 256


def _group_rank(group) -> Tuple[int, int]:
    if not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _allgather_obj(obj, group):
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [obj]
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


class SymmetricHeap:
    """One IPC-mapped heap per rank; see the module docstring."""

    DEFAULT_BYTES = int(os.environ.get("DGRAPH_SYMHEAP_BYTES", str(1 << 30)))

    def __init__(self, nbytes: int, group=None, device: Optional[torch.device] = None):
        self.group = group
        self.rank, self.world = _group_rank(group)
        dev = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.device = dev
        ops = _native.ops()
        sizes = _allgather_obj(int(nbytes), group)
        self.nbytes = (max(sizes) + _ALIGN - 1) // _ALIGN * _ALIGN
        self.local = ops.heap_alloc(self.nbytes, dev.index)
        handle = ops.ipc_get_handle(self.local)
        handles = _allgather_obj(bytes(handle.numpy().tobytes()), group)
        self._opened = []
        ptrs = []
        for p, hb in enumerate(handles):
            if p == self.rank:
                ptrs.append(ops.tensor_ptr(self.local))
            else:
                h = torch.frombuffer(bytearray(hb), dtype=torch.uint8)
                ptr = ops.ipc_open_handle(h, dev.index)
                self._opened.append(ptr)
                ptrs.append(ptr)
        self.peer_ptrs = ptrs
        self.table = torch.tensor(ptrs, dtype=torch.int64, device=dev)
        self._cursor = 0
        self._allocs: Dict[int, Tuple[int, int]] = {}  # data_ptr -> (offset, nbytes)
        self._put_cache: Dict[tuple, Tuple[torch.Tensor, torch.Tensor]] = {}
        self.barrier()

    # ------------------------------------------------------------------ lifecycle
    @classmethod
    def create(cls, group=None, nbytes: Optional[int] = None) -> "SymmetricHeap":
        return cls(nbytes or cls.DEFAULT_BYTES, group)

    def close(self) -> None:
        if self.local is None:
            return
        torch.cuda.synchronize(self.device)
        self.barrier()
        ops = _native.ops()
        for ptr in self._opened:
            ops.ipc_close(ptr)
        self._opened = []
        self.local = None
        self.table = None

    def barrier(self) -> None:
        """All prior heap traffic of every rank is complete and visible."""
        if self.local is not None and self.local.is_cuda:
            torch.cuda.current_stream(self.device).synchronize()
        if dist.is_initialized() and self.world > 1:
            dist.barrier(group=self.group)

    # ------------------------------------------------------------------ allocation
    def alloc_tensor(self, size, dtype: torch.dtype) -> torch.Tensor:
        """Carve a symmetric tensor (collective by convention: same call order on all ranks)."""
        shape = tuple(size) if isinstance(size, Sequence) else (int(size),)
        n = 1
        for s in shape:
            n *= int(s)
        es = torch.empty((), dtype=dtype).element_size()
        nb = n * es
        off = (self._cursor + _ALIGN - 1) // _ALIGN * _ALIGN
        if off + nb > self.nbytes:
            raise MemoryError(f"symmetric heap exhausted: need {off + nb} of {self.nbytes} bytes "
                              "(set DGRAPH_SYMHEAP_BYTES)")
        self._cursor = off + nb
        t = self.local[off:off + nb].view(dtype).view(shape)
        self._allocs[t.data_ptr()] = (off, nb)
        return t

    def reset(self) -> None:
        """Release every symmetric tensor (collective)."""
        self._cursor = 0
        self._allocs.clear()
        self._put_cache.clear()

    def owns(self, t: torch.Tensor) -> bool:
        if self.local is None or not t.is_cuda or t.device != self.local.device:
            return False
        base = self.local.data_ptr()
        return base <= t.data_ptr() < base + self.nbytes

    def offset_of(self, t: torch.Tensor) -> int:
        if not self.owns(t):
            raise ValueError("tensor is not on the symmetric heap")
        return t.data_ptr() - self.local.data_ptr()

    # ------------------------------------------------------------------ one-sided ops
    def remote_gather(self, x: torch.Tensor, indices: torch.Tensor,
                      owners: torch.Tensor) -> torch.Tensor:
        """``out[i] = x_on_rank[owners[i]][indices[i]]`` — the local-form G1 gather.

        ``x`` ([N_r, F], per-rank row counts may differ) is staged into a symmetric slot
        sized for the largest N_r, then every output row is fetched straight from its
        owner's heap.
        """
        F = x.shape[-1]
        x2 = x.reshape(-1, F)
        n_max = max(_allgather_obj(int(x2.shape[0]), self.group))
        mark = self._cursor
        stage = self.alloc_tensor((max(n_max, 1), F), x2.dtype)
        stage[: x2.shape[0]].copy_(x2)
        self.barrier()  # every rank has staged its rows
        out = torch.empty(indices.numel(), F, dtype=x2.dtype, device=x2.device)
        if out.numel():
            _native.ops().heap_get_rows(self.table, self.offset_of(stage),
                                        owners.reshape(-1).long().contiguous(),
                                        indices.reshape(-1).long().contiguous(), out, F)
        self.barrier()  # nobody reuses the staging slot while peers still read it
        self._release_to(mark)
        return out

    def put_rows(self, send: torch.Tensor, recv: torch.Tensor, send_splits: Sequence[int],
                 remote_offsets: Sequence[int]) -> None:
        """Rows ``send[so_p : so_p + n_p]`` land in peer ``p``'s ``recv`` at row
        ``remote_offsets[p]`` (``recv`` must be a symmetric tensor). Synchronous."""
        F = send.shape[-1]
        s2 = send.reshape(-1, F).contiguous()
        key = (tuple(int(v) for v in send_splits), tuple(int(v) for v in remote_offsets))
        idx = self._put_cache.get(key)
        if idx is None:
            peers = torch.repeat_interleave(torch.arange(len(key[0])),
                                            torch.tensor(key[0], dtype=torch.long))
            starts = torch.tensor(key[1], dtype=torch.long)
            so = torch.cumsum(torch.tensor((0,) + key[0][:-1], dtype=torch.long), 0)
            pos = torch.arange(peers.numel()) - so[peers] + starts[peers]
            idx = (peers.to(s2.device), pos.to(s2.device))
            self._put_cache[key] = idx
        if s2.shape[0]:
            _native.ops().heap_put_rows(self.table, self.offset_of(recv), idx[0], idx[1], s2,
                                        recv.reshape(-1, F).stride(0))
        self.barrier()

    def _release_to(self, mark: int) -> None:
        self._cursor = mark
        for p in [p for p, (o, _) in self._allocs.items() if o >= mark]:
            del self._allocs[p]


class NVSHMEMP2P:
    """API-compatible facade of the reference's ``torch_nvshmem_p2p.NVSHMEMP2P``
    (torch_nvshmem_p2p_bindings.cpp:19-36) on top of :class:`SymmetricHeap`."""

    _heap: Optional[SymmetricHeap] = None

    @staticmethod
    def init(group=None, nbytes: Optional[int] = None) -> None:
        if NVSHMEMP2P._heap is None:
            NVSHMEMP2P._heap = SymmetricHeap.create(group, nbytes)

    @staticmethod
    def _h() -> SymmetricHeap:
        if NVSHMEMP2P._heap is None:
            NVSHMEMP2P.init()
        return NVSHMEMP2P._heap

    @staticmethod
    def finalize() -> None:
        if NVSHMEMP2P._heap is not None:
            NVSHMEMP2P._heap.close()
            NVSHMEMP2P._heap = None

    @staticmethod
    def get_rank() -> int:
        return NVSHMEMP2P._h().rank

    @staticmethod
    def get_world_size() -> int:
        return NVSHMEMP2P._h().world

    @staticmethod
    def allocate_symmetric_memory(num_elem: int, device_index: int = 0,
                                  dtype: torch.dtype = torch.float32) -> torch.Tensor:
        return NVSHMEMP2P._h().alloc_tensor((int(num_elem),), dtype)

    @staticmethod
    def clone_tensor(t: torch.Tensor) -> torch.Tensor:
        out = NVSHMEMP2P._h().alloc_tensor(tuple(t.shape), t.dtype)
        out.copy_(t)
        return out

    @staticmethod
    def padded_clone_tensor(t: torch.Tensor, num_elem: int) -> torch.Tensor:
        out = NVSHMEMP2P._h().alloc_tensor((int(num_elem),), t.dtype)
        out.zero_()
        out[: t.numel()].copy_(t.reshape(-1))
        return out

    @staticmethod
    def register_memory(t: torch.Tensor) -> None:  # heap memory is always registered
        return None

    @staticmethod
    def deregister_memory(t: torch.Tensor) -> None:
        return None

    @staticmethod
    def dist_get(src, dst, indices, rank_mappings, bs, num_input_rows, num_features,
                 num_output_rows) -> None:
        """``dst[0, i] = src_on[rank_mappings[i]][0, indices[i]]`` (batch size 1)."""
        assert int(bs) == 1, "batch size must be 1"
        out = NVSHMEMP2P._h().remote_gather(src.reshape(-1, int(num_features)),
                                            indices.reshape(-1), rank_mappings.reshape(-1))
        dst.reshape(-1, int(num_features))[: out.shape[0]].copy_(out)

    @staticmethod
    def get_max(val: int) -> int:
        h = NVSHMEMP2P._h()
        return max(_allgather_obj(int(val), h.group))

    @staticmethod
    def barrier() -> None:
        NVSHMEMP2P._h().barrier()

    @staticmethod
    def barrier_stream() -> None:
        NVSHMEMP2P._h().barrier()
