"""Symmetric device heap over HIP IPC — the one-sided transport of the ``rocshmem`` /
``nvshmem`` backend (replaces NVSHMEM: DGraph/distributed/csrc/torch_nvshmem_p2p.cu:32-376,
nvshmem_comm_kernels.cuh:60-170).

Every rank of the group ``hipMalloc``'s one heap of the same size (the max of the requested
sizes — the reference's collective ``nvshmem_malloc`` was called with per-rank sizes, D4),
publishes its IPC handle, and maps every peer heap. Tensors carved from the heap with
:meth:`SymmetricHeap.alloc_tensor` live at the same offset on every rank (allocation is a
collective bump allocator: all ranks allocate in the same order), so a peer's copy of a
symmetric tensor is ``peer_base[p] + offset``. Native kernels (csrc/comm/symheap.hip) then

* read remote rows directly over xGMI (:meth:`remote_gather`, the K15 ``dist_get``),
* write rows into peers' receive buffers at ``remote_offsets`` (:meth:`put_rows`), and
* scatter-add rows into peers' symmetric outputs (:meth:`scatter_add`, the ``dist_put`` of
  torch_nvshmem_p2p.cu:96-164) — deterministically: each rank pre-aggregates its rows per
  (destination rank, row), puts the partial sums into a per-source slot of the owner's
  heap, and the owner adds the slots with a fixed-order segment sum (no float atomics; the
  reference's CAS loop made the sum order, and so the bits, run-dependent).

Completion is STREAM-ORDERED and device-side (no host sync on the data path; the
reference used nvshmemx_quiet_on_stream / barrier_all_on_stream, torch_nvshmem_p2p.cu:
149,162,366-376): the heap starts with flag words, a producer kernel is followed on the
same stream by ``heap_signal`` (system-scope release of a monotonic epoch into every peer's
flag) and a consumer waits with ``heap_wait`` (system-scope acquire spin, bounded).
:meth:`barrier_stream` is the device-side barrier; :meth:`barrier` additionally drains the
host (start-up / tear-down only). Tensors gathered repeatedly are registered once
(:meth:`register`: a persistent heap copy, refreshed when the tensor's version changes), so
the steady state has no per-call negotiation, staging allocation or host barrier.
"""
from __future__ import annotations

import os
import weakref
from typing import Dict, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import _native

_ALIGN = 256
# flag words at the start of every heap: kind k, source rank q -> word k * 64 + q
_MAX_W = 64
_READY, _DONE, _BAR, _PUT, _PUTDONE, _SC, _SCDONE = range(7)
_NKINDS = 8
_FLAG_BYTES = _NKINDS * _MAX_W * 8
_MAX_SPINS = int(os.environ.get("DGRAPH_SHMEM_MAX_SPINS", str(1 << 23)))  # ~10 s bound


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


def _base_of(t: torch.Tensor) -> torch.Tensor:
    return t._base if t._base is not None else t


def _view_key(t: torch.Tensor) -> tuple:
    """Identity of the data a tensor (or any view object of it) denotes: its base tensor,
    storage offset, shape, strides and dtype. Two view objects of the same data share the
    key, so per-call ``x[0]`` / ``reshape`` views hit the cache; the base identity is
    verified through a weak reference at lookup (a freed base's id can be reused)."""
    return (id(_base_of(t)), t.storage_offset(), tuple(t.shape), tuple(t.stride()), t.dtype)


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
        # DGRAPH_SYMHEAP_FINE=1: fine-grained device memory (see csrc/comm/comm_ops.cpp
        # heap_alloc); default coarse-grained hipMalloc
        self.fine = os.environ.get("DGRAPH_SYMHEAP_FINE", "0") == "1"
        self.local = ops.heap_alloc(self.nbytes, dev.index, self.fine)
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
        if self.world > _MAX_W:
            raise ValueError(f"symmetric heap supports up to {_MAX_W} ranks per group")
        # flag words (zeroed before any peer can signal: the init barrier below)
        self.flags = self.local[:_FLAG_BYTES].view(torch.int64).view(_NKINDS, _MAX_W)
        self.flags.zero_()
        self._epoch = [0] * _NKINDS
        # timeout word of the device-side waits: pinned host memory, so check() is a plain
        # host load that every data-path call can afford (a device word would need a sync)
        try:
            self._timed_out = torch.zeros(1, dtype=torch.int32).pin_memory() \
                if dev.type == "cuda" else torch.zeros(1, dtype=torch.int32)
        except RuntimeError:
            self._timed_out = torch.zeros(1, dtype=torch.int32, device=dev)
        self._cursor = _FLAG_BYTES
        self._allocs: Dict[int, Tuple[int, int]] = {}  # data_ptr -> (offset, nbytes)
        self._put_cache: Dict[tuple, Tuple[torch.Tensor, torch.Tensor]] = {}
        self._registered: Dict[tuple, dict] = {}  # view key -> registration
        self._scatter_plans: Dict[tuple, "_ScatterPlan"] = {}
        # Device-side completion needs every rank's kernels to run concurrently (one GPU
        # per rank). Ranks sharing one GPU (the 2-process-on-one-GPU test harness) are
        # time-sliced between processes, so a spinning wait could starve the peer whose
        # signal it awaits: such groups complete through the host instead (same data
        # path, host barriers). DGRAPH_SHMEM_COMPLETION=device|host overrides.
        mode = os.environ.get("DGRAPH_SHMEM_COMPLETION", "auto")
        if mode == "auto":
            uid = str(getattr(torch.cuda.get_device_properties(dev), "uuid", "")) \
                if dev.type == "cuda" else ""
            ids = _allgather_obj((os.uname().nodename, uid, dev.index), group)
            mode = "host" if len(set(ids)) < len(ids) else "device"
        self.device_completion = mode == "device"
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
        """Host-level: all prior heap traffic of every rank is complete and visible
        (start-up / tear-down; the data path uses :meth:`barrier_stream`)."""
        if self.local is not None and self.local.is_cuda:
            # the whole device, not the current stream: heap traffic (a copy-out of a
            # receive slot) may have been enqueued on the comm side stream or on the
            # compute stream, depending on the caller
            torch.cuda.synchronize(self.device)
            self.check()
        if dist.is_initialized() and self.world > 1:
            dist.barrier(group=self.group)

    # ------------------------------------------------------------------ device completion
    def _flag_off(self, kind: int) -> int:
        return kind * _MAX_W * 8

    def signal(self, kind: int, epoch: int, self_too: bool = False) -> None:
        """Stream-ordered: after this stream's earlier kernels, store ``epoch`` into
        ``flags[kind][me]`` of every peer's heap (system-scope release)."""
        if self.world > 1 or self_too:
            _native.ops().heap_signal(self.table, self._flag_off(kind), self.rank,
                                      self.world, int(epoch), bool(self_too))

    def wait(self, kind: int, epoch: int, self_too: bool = False) -> None:
        """Stream-ordered: later kernels on this stream start once every peer q has
        signalled ``flags[kind][q] >= epoch`` (bounded spin; see :meth:`check`)."""
        if self.world > 1 or self_too:
            _native.ops().heap_wait(self.flags[kind], self.rank, self.world, int(epoch),
                                    _MAX_SPINS, bool(self_too), self._timed_out)

    def next_epoch(self, kind: int) -> int:
        self._epoch[kind] += 1
        return self._epoch[kind]

    def barrier_stream(self) -> None:
        """Device-side barrier of the group (nvshmemx_barrier_all_on_stream): no host sync;
        the stream proceeds once every peer's stream reached its barrier_stream."""
        if not self.device_completion:
            self.barrier()
            return
        e = self.next_epoch(_BAR)
        self.signal(_BAR, e)
        self.wait(_BAR, e)

    def check(self) -> None:
        """Raise if a device-side wait gave up (a peer never signalled). The flag is a
        pinned host word written by the wait kernel: reading it does not sync the device,
        so every data-path call checks it on entry (a timeout in call k is reported by call
        k + 1 at the latest, or by the next :meth:`barrier`)."""
        t = self._timed_out
        if t is None:
            return
        v = int(t[0]) if not t.is_cuda else int(t.item())
        if v != 0:
            raise RuntimeError("symmetric heap: a device-side wait timed out (a peer did not "
                               "reach the matching signal; see DGRAPH_SHMEM_MAX_SPINS)")

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
        self._cursor = _FLAG_BYTES
        self._allocs.clear()
        self._put_cache.clear()
        self._registered.clear()
        self._scatter_plans.clear()

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
    def register(self, x: torch.Tensor) -> torch.Tensor:
        """Collective (first call for a tensor): a persistent symmetric copy of ``x``
        ([N_r, F], per-rank N may differ; the slot is sized for the largest). Later
        :meth:`remote_gather` calls on the same data — the same tensor or any view object
        of it with the same offset, shape and strides (callers pass fresh ``x[0]`` /
        ``reshape`` views every call) — reuse it; an in-place update (version change) is
        re-copied into the same slot without renegotiation. Slots of registrations whose
        tensor has been freed ON EVERY RANK are reused (agreed collectively, so a slot
        sits at the same heap offset everywhere)."""
        F = x.shape[-1]
        x2 = x.reshape(-1, F)
        es = x2.element_size()
        dead = sorted((e["slot"].data_ptr() - self.local.data_ptr(), e["slot"].numel() * es, k)
                      for k, e in self._registered.items() if e["ref"]() is None)
        infos = _allgather_obj((int(x2.shape[0]), [(o, n) for o, n, _ in dead]), self.group)
        n_max = max(i[0] for i in infos)
        need = max(n_max, 1) * F * es
        common = set.intersection(*[set(map(tuple, i[1])) for i in infos])
        slot = None
        for off, nb, k in dead:
            if (off, nb) in common and nb >= need:
                del self._registered[k]
                slot = self.local[off:off + need].view(x2.dtype).view(max(n_max, 1), F)
                break
        if slot is None:
            slot = self.alloc_tensor((max(n_max, 1), F), x2.dtype)
        elif self.device_completion:
            # a reused slot: peers' reads of its previous tensor (a remote_gather of the last
            # epoch, still running on their GPUs) must be done before it is overwritten —
            # the same write-after-read wait as the version-change path of _slot_for
            self.wait(_DONE, self._epoch[_DONE])
        slot[: x2.shape[0]].copy_(x2)
        base = x._base if x._base is not None else x
        ent = {"ref": weakref.ref(base), "version": x._version, "slot": slot,
               "rows": x2.shape[0]}
        self._registered[_view_key(x)] = ent
        return slot

    def _slot_for(self, x: torch.Tensor) -> torch.Tensor:
        if self.owns(x):
            return x.reshape(-1, x.shape[-1])
        ent = self._registered.get(_view_key(x))
        base = x._base if x._base is not None else x
        if ent is None or ent["ref"]() is not base:
            return self.register(x)
        if ent["version"] != x._version:
            # readers of the previous epoch must be done with the slot before it changes
            if self.device_completion:
                self.wait(_DONE, self._epoch[_DONE])
            ent["slot"][: ent["rows"]].copy_(x.reshape(-1, x.shape[-1]))
            ent["version"] = x._version
        return ent["slot"]

    def remote_gather(self, x: torch.Tensor, indices: torch.Tensor,
                      owners: torch.Tensor) -> torch.Tensor:
        """``out[i] = x_on_rank[owners[i]][indices[i]]`` — the local-form G1 gather.

        Stream-ordered one-sided get: every rank publishes its (registered or heap-resident)
        rows with a READY signal, waits for its peers' READY, reads the rows straight from
        the owners' heaps over xGMI, and releases the slots with a DONE signal. No host
        synchronisation after the first (registering) call for a tensor.
        """
        F = x.shape[-1]
        self.check()
        slot = self._slot_for(x)
        if self.device_completion:
            e = self.next_epoch(_READY)
            self.signal(_READY, e)
            self.wait(_READY, e)
        else:
            self.barrier()  # every owner has (re)written its slot
        out = torch.empty(indices.numel(), F, dtype=x.dtype, device=x.device)
        if out.numel():
            _native.ops().heap_get_rows(self.table, self.offset_of(slot),
                                        owners.reshape(-1).long().contiguous(),
                                        indices.reshape(-1).long().contiguous(), out,
                                        slot.stride(0))
        if self.device_completion:
            d = self.next_epoch(_DONE)
            self.signal(_DONE, d)
            if self.owns(x):
                # peers read a heap-resident x in place (no private slot): later kernels on
                # this stream — which may overwrite x, e.g. with the next layer's output —
                # start only once every peer has finished reading it (write-after-read)
                self.wait(_DONE, d)
        else:
            self.barrier()  # nobody rewrites a slot while peers still read it
        return out

    def put_rows(self, send: torch.Tensor, recv: torch.Tensor, send_splits: Sequence[int],
                 remote_offsets: Sequence[int]) -> None:
        """Rows ``send[so_p : so_p + n_p]`` land in peer ``p``'s ``recv`` at row
        ``remote_offsets[p]`` (``recv`` must be a symmetric tensor). Stream-ordered:
        kernels issued after this call on the current stream see every peer's rows in
        ``recv``; a peer's rows of the previous call are not overwritten before that peer
        has entered this call (its reads of them were issued before)."""
        F = send.shape[-1]
        self.check()
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
        if not self.device_completion:
            self.barrier()
            if s2.shape[0]:
                _native.ops().heap_put_rows(self.table, self.offset_of(recv), idx[0], idx[1],
                                            s2, recv.reshape(-1, F).stride(0))
            self.barrier()
            return
        # the previous epoch's receivers are done with their recv (they entered this call)
        prev = self._epoch[_PUT]
        self.signal(_PUTDONE, prev)
        self.wait(_PUTDONE, prev)
        if s2.shape[0]:
            _native.ops().heap_put_rows(self.table, self.offset_of(recv), idx[0], idx[1], s2,
                                        recv.reshape(-1, F).stride(0))
        e = self.next_epoch(_PUT)
        self.signal(_PUT, e)
        self.wait(_PUT, e)  # every peer's rows have landed in my recv

    def scatter_add(self, x: torch.Tensor, indices: torch.Tensor, owners: torch.Tensor,
                    num_output_rows: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One-sided scatter-add (the reference's ``dist_put``):
        ``out_on_rank[owners[i]][indices[i]] += x[i]``; returns this rank's ``out``
        ([num_output_rows, F], zero-initialised when not given).

        Deterministic: rows are pre-summed locally per (owner, row), put as one block per
        owner into this rank's slot range of the owner's symmetric receive area, and every
        owner adds its slots with a fixed-order segment sum. The plan (slot layout and the
        owners' segment-sum CSR) is built once per index tensor pair — collectively, so all
        ranks must pass their index tensors consistently (same objects, unmodified) to hit
        it — after which a call is two local SpMMs, one put kernel and the completion
        signals: no host synchronisation."""
        from ..ops import kernels as K

        F = x.shape[-1]
        x2 = x.reshape(-1, F).contiguous()
        plan = self._scatter_plan(indices, owners, int(num_output_rows), F, x2.dtype)
        if out is None:
            out = torch.zeros(int(num_output_rows), F, dtype=x2.dtype, device=x2.device)
        agg = K.spmm(plan.pre.rowptr, plan.pre.col, x2) if plan.pre.nnz else \
            x2.new_zeros(0, F)
        self.put_rows(agg, plan.slot, plan.send_splits, plan.remote_offsets)
        post = plan.post
        if post.nnz:
            o2 = out.reshape(-1, F)
            K.spmm(post.rowptr, post.col, plan.slot, o2, beta=1.0, row_map=post.row_map)
        return out

    def _scatter_plan(self, indices, owners, n_out: int, F: int, dtype) -> "_ScatterPlan":
        # keyed by the index DATA (base tensor, offset, shape, strides), not the Python view
        # object: engines pass a fresh ``indices.reshape(-1)`` every call
        key = (_view_key(indices), _view_key(owners), n_out, F, dtype)
        plan = self._scatter_plans.get(key)
        if plan is not None and plan.matches(indices, owners):
            return plan
        # drop plans whose index tensors are gone (their slots stay allocated: bump heap)
        for k in [k for k, p in self._scatter_plans.items() if p.dead()]:
            del self._scatter_plans[k]
        plan = _ScatterPlan(self, indices, owners, n_out, F, dtype)
        self._scatter_plans[key] = plan
        return plan

    def _release_to(self, mark: int) -> None:
        self._cursor = mark
        for p in [p for p, (o, _) in self._allocs.items() if o >= mark]:
            del self._allocs[p]


class _ScatterPlan:
    """Slot layout of one :meth:`SymmetricHeap.scatter_add` pattern (built collectively)."""

    def __init__(self, heap: SymmetricHeap, indices, owners, n_out: int, F: int, dtype):
        from ..ops.csr import CSR
        from ..plan.pattern import _alltoall_counts, _alltoallv_ids

        self.refs = (weakref.ref(_base_of(indices)), weakref.ref(_base_of(owners)))
        self.versions = (indices._version, owners._version)
        dev = heap.device
        W = heap.world
        idx = indices.reshape(-1).to(dev).long()
        dst = owners.reshape(-1).to(dev).long()
        n = idx.numel()
        # (owner, row) key: rows index the OWNER's output, so the radix is this rank's
        # largest target row + 1 (not its own n_out)
        M = int(idx.max().item()) + 1 if n else 1
        key = dst * M + idx
        uniq, inv = (torch.unique(key, sorted=True, return_inverse=True) if n else
                     (key, key))
        U = uniq.numel()
        # local pre-aggregation: unique (owner, row) u <- the input rows that target it
        self.pre = CSR.from_coo(inv, torch.arange(n, device=dev), U, max(n, 1))
        udst = torch.div(uniq, M, rounding_mode="floor")
        uidx = uniq - udst * M
        counts = torch.bincount(udst, minlength=W) if U else torch.zeros(W, dtype=torch.long,
                                                                          device=dev)
        group = heap.group
        peer_counts = _alltoall_counts(counts, group) if W > 1 else counts.clone()
        self.send_splits = [int(v) for v in counts.tolist()]
        recv_splits = [int(v) for v in peer_counts.tolist()]
        recv_idx = _alltoallv_ids(uidx, self.send_splits, recv_splits, group) if W > 1 \
            else uidx
        R = sum(recv_splits)
        r_max = max(_allgather_obj(R, group))
        # my rows land in owner p's slots at p's prefix over its sources
        prefix = torch.zeros(W, dtype=torch.long, device=dev)
        if W > 1:
            prefix[1:] = torch.cumsum(peer_counts, 0)[:-1]
            remote = _alltoall_counts(prefix, group)
        else:
            remote = prefix
        self.remote_offsets = [int(v) for v in remote.tolist()]
        self.slot = heap.alloc_tensor((max(r_max, 1), F), dtype)
        # owner side: output row <- slot positions, source-major (fixed summation order)
        self.post = CSR.from_coo(recv_idx.to(dev).long(), torch.arange(R, device=dev), n_out,
                                 max(r_max, 1)).compact_rows()

    def matches(self, indices, owners) -> bool:
        return (self.refs[0]() is _base_of(indices) and self.refs[1]() is _base_of(owners)
                and self.versions == (indices._version, owners._version))

    def dead(self) -> bool:
        return self.refs[0]() is None or self.refs[1]() is None


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
    def dist_put(src, dst, indices, rank_mappings, bs, num_input_rows, num_features,
                 num_output_rows) -> None:
        """``dst_on[rank_mappings[i]][0, indices[i]] += src[0, i]`` (batch size 1); ``dst``
        is this rank's output (symmetric or not). Deterministic one-sided scatter-add
        (:meth:`SymmetricHeap.scatter_add`), stream-ordered."""
        assert int(bs) == 1, "batch size must be 1"
        F = int(num_features)
        out = dst.reshape(-1, F)[: int(num_output_rows)]
        NVSHMEMP2P._h().scatter_add(src.reshape(-1, F)[: int(num_input_rows)],
                                    indices.reshape(-1)[: int(num_input_rows)],
                                    rank_mappings.reshape(-1)[: int(num_input_rows)],
                                    int(num_output_rows), out=out)

    @staticmethod
    def get_max(val: int) -> int:
        h = NVSHMEMP2P._h()
        return max(_allgather_obj(int(val), h.group))

    @staticmethod
    def barrier() -> None:
        NVSHMEMP2P._h().barrier()

    @staticmethod
    def barrier_stream() -> None:
        """Device-side barrier on the current stream (no host sync)."""
        NVSHMEMP2P._h().barrier_stream()
