"""All-to-all-v executor with host-cached split vectors.

The reference recomputes split lists from device tensors on every call
(``_get_splits`` ``.tolist()`` x2 at NCCLBackendEngine.py:257-274, one device sync per
halo exchange). Plans here are static (I6), so the splits are turned into Python lists
once and the exchange is a single stream-ordered RCCL all-to-all-v: every peer pair
(i -> j) rides its own xGMI link, all 7 links concurrently. ``async_op=True`` returns a
handle whose ``wait()`` only makes the *current stream* wait (no host sync), which is
what the interior/boundary overlap in :mod:`dgraph_amd.parallel.dist_graph` builds on.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

# Transport of the halo all-to-all-v. Default "torch": ProcessGroupNCCL, i.e. RCCL through
# torch.distributed on a high-priority stream (comm/groups.py). Decision (round 2): both
# paths issue the same RCCL grouped send/recv kernels over the same xGMI links, so the
# data movement is identical; the PG path additionally carries the NCCL watchdog /
# timeout / async error handling that failure detection (§5.3) relies on, costs no
# second communicator (RCCL buffers per peer and channel), and is the one exercised by
# the W = 2..8 equivalence tests. "native" (comm/rccl_exec.py: a private communicator,
# several tensors per group call, completion as a HIP event) stays selectable with
# DGRAPH_A2A_IMPL=native for A/B runs on a multi-GPU node (benchmarks/bench_comm.py).
#
# "shmem": one-sided puts into the receivers' symmetric-heap slots over xGMI
# (comm/symheap.py; the reference's put contract with remote offsets,
# DGraph/distributed/Engine.py:67-86, commInfo.py:205-206). Needs no RCCL communicator, so it
# also runs ranks that share one GPU (RCCL refuses two ranks per device): the
# 2-process-on-one-GPU equivalence test of the bench step uses it.
A2A_IMPL = os.environ.get("DGRAPH_A2A_IMPL", "torch")

# Link model of the LOOPBACK exchange (a W-way plan run by one process: bench.py
# --rehearse-world). 0 = the copy completes at once (a loopback exposes nothing). > 0: the
# copy is issued on a side stream as one kernel of LOOPBACK_CUS workgroups that takes at
# least latency + max-per-peer-bytes / (GBPS * 1e9) — each peer message rides its own link,
# all links concurrently — and the call returns a PENDING work whose wait() is a stream
# event wait, so the executor's overlap schedule meets a link-length transfer and its
# exposed-exchange regions measure what a W-GPU run would expose (the reference timed its
# exchange regions separately, experiments/OGB/GCN.py:101-116).
LOOPBACK_LINK_GBPS = float(os.environ.get("DGRAPH_LOOPBACK_LINK_GBPS", "0"))
LOOPBACK_LATENCY_US = float(os.environ.get("DGRAPH_LOOPBACK_LATENCY_US", "15"))
# CUs the modelled collective's kernel holds while the transfer runs (one wave each): RCCL
# moves an all-to-all with one workgroup per channel, each resident on a CU for the whole
# transfer; a block of another kernel that needs the whole CU (the fp32 GEMM) cannot start
# there until it ends
LOOPBACK_CUS = int(os.environ.get("DGRAPH_LOOPBACK_CUS", "16"))
# workgroups that move the modelled transfer's bytes — its HBM traffic at both ends (a
# real rank reads what it sends and has what it receives written): enough for a full-rate
# copy, which leaves the CUs again well within the link time (64 workgroups, ~1/4 of the
# CUs, copied a W=8 rank's 24 GB column block at ~0.5 TB/s and held those CUs for twice
# the link time, profiles/r05/); the first LOOPBACK_CUS of them then stay until the link
# time has passed
LOOPBACK_COPY_CUS = int(os.environ.get("DGRAPH_LOOPBACK_COPY_CUS", "1024"))

_HEAPS: dict = {}


def shmem_heap(group, device):
    """The process-wide symmetric heap of ``group`` on ``device`` (created collectively on
    first use; size DGRAPH_SYMHEAP_BYTES)."""
    key = (id(group), str(device))
    h = _HEAPS.get(key)
    if h is None:
        from .symheap import SymmetricHeap

        h = SymmetricHeap(SymmetricHeap.DEFAULT_BYTES, group, device)
        _HEAPS[key] = h
    return h


def close_shmem_heaps() -> None:
    for h in _HEAPS.values():
        h.close()
    _HEAPS.clear()


def offsets_to_splits(offsets) -> List[int]:
    if isinstance(offsets, torch.Tensor):
        o = offsets.detach().cpu().tolist()
    else:
        o = list(offsets)
    return [int(o[i + 1] - o[i]) for i in range(len(o) - 1)]


class _Done:
    def wait(self):
        return None

    def is_completed(self):
        return True


class _EventWork:
    """A pending exchange completed by a stream event: ``wait()`` makes the CURRENT stream
    wait for it (no host synchronisation). ``keep``: the tensors the exchange's stream still
    uses, held until ``wait()`` instead of ``record_stream`` — a block freed with a pending
    use on another stream cannot be reused until the allocator sees that stream's work done,
    so every exchange of a step allocated fresh memory, and near the HBM limit the
    allocator's retry (free the whole cache, synchronise) stalled the host for seconds (an
    R-GCN rehearsal rank: 21 hipMallocs and 2 retries in 2 steps, 2.6 s of idle GPU per step,
    profiles/r05/). After ``wait()`` the waiting stream is ordered after the exchange, so
    the blocks are free for its work (the TORCH_NCCL_AVOID_RECORD_STREAMS scheme)."""

    def __init__(self, event, keep=()):
        self.event = event
        self.keep = keep

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)
        self.keep = ()
        return None

    def is_completed(self):
        return self.event.query()


def _stream_done(t: torch.Tensor):
    """Completion of work just enqueued on the CURRENT stream (which may be a comm side
    stream, not the caller's compute stream): an event recorded there, so ``wait()`` orders
    whichever stream is current at wait time after it. The contract every transport keeps:
    a returned work's ``wait()`` orders the waiting stream after ALL device work the call
    enqueued, on any stream (the reference's put was synchronous,
    DGraph/distributed/Engine.py:67-86, and its halo buffer was consumed only after it
    returned, haloExchange.py:47-62). Host-only tensors complete at once."""
    if not t.is_cuda:
        return _Done()
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    return _EventWork(ev)


_SIDE: dict = {}


def _side_stream(dev) -> "torch.cuda.Stream":
    """The communication stream of ``dev``: HIGH priority. Streams map onto a handful of
    hardware queues, and a stream that lands on the compute stream's queue runs in order
    with it — no overlap at all (a W=8 rehearsal's kernel trace had both on one queue,
    profiles/r05/timeline_w8_structureless_shared_queue.txt); high-priority streams sit on
    queues of their own (scripts/debug/queue_probe.py), and the exchange's kernels are the
    ones to dispatch first (RCCL's own streams are high priority too)."""
    s = _SIDE.get(dev.index)
    if s is None:
        s = torch.cuda.Stream(dev, priority=-1)
        _SIDE[dev.index] = s
    return s


class CommStats:
    """Process-wide byte counters (plan statistics / metrics stream)."""

    calls = 0
    bytes_sent = 0
    bytes_recv = 0
    peer_bytes_sent: dict = {}  # group-local peer rank -> bytes sent to it

    @classmethod
    def reset(cls):
        cls.calls = cls.bytes_sent = cls.bytes_recv = 0
        cls.peer_bytes_sent = {}


class AllToAllV:
    """Exchange rows: rank r sends ``send[send_off[p]:send_off[p+1]]`` to peer p and
    receives peer q's segment into ``recv[recv_off[q]:recv_off[q+1]]``."""

    def __init__(self, send_splits: Sequence[int], recv_splits: Sequence[int],
                 group: Optional[dist.ProcessGroup] = None):
        self.send_splits = [int(s) for s in send_splits]
        self.recv_splits = [int(s) for s in recv_splits]
        self.group = group
        self.total_send = sum(self.send_splits)
        self.total_recv = sum(self.recv_splits)
        self._world = len(self.send_splits)
        self._shm_offsets = None  # peers' receive offsets of my rows (shmem transport)
        self._shm_slots: dict = {}  # (row shape, dtype) -> symmetric receive slot

    def reversed(self) -> "AllToAllV":
        return AllToAllV(self.recv_splits, self.send_splits, self.group)

    def __call__(self, send: torch.Tensor, out: Optional[torch.Tensor] = None,
                 async_op: bool = False):
        if send.shape[0] != self.total_send:
            raise ValueError(f"send has {send.shape[0]} rows, plan expects {self.total_send}")
        if out is None:
            out = torch.empty((self.total_recv,) + tuple(send.shape[1:]), dtype=send.dtype,
                              device=send.device)
        row_bytes = send[0:1].numel() * send.element_size() if send.dim() > 0 else send.element_size()
        CommStats.calls += 1
        CommStats.bytes_sent += self.total_send * row_bytes
        CommStats.bytes_recv += self.total_recv * row_bytes
        pb = CommStats.peer_bytes_sent
        for p, n in enumerate(self.send_splits):
            if n:
                pb[p] = pb.get(p, 0) + n * row_bytes
        from .faults import FaultInjector

        if FaultInjector.active():
            send = FaultInjector.before_exchange(
                send, dist.get_rank() if dist.is_initialized() else 0)
        if self._world <= 1 or not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return self._loopback(send, out, row_bytes, async_op)
        send_c = send.contiguous()
        if A2A_IMPL == "shmem" and send_c.is_cuda:
            work = self._shmem(send_c, out, async_op)
            if async_op:
                return out, work
            work.wait()
            return out
        if A2A_IMPL == "native" and send_c.is_cuda:
            from .rccl_exec import RCCLExecutor

            work = RCCLExecutor.for_group(self.group).alltoallv(
                [send_c], [out], self.send_splits, self.recv_splits, async_op=async_op)
            return (out, work) if async_op else out
        work = dist.all_to_all_single(
            out, send_c,
            output_split_sizes=self.recv_splits,
            input_split_sizes=self.send_splits,
            group=self.group,
            async_op=async_op,
        )
        if async_op:
            return out, work
        return out


    def link_us(self, row_bytes: int, gbps: float = 0.0) -> float:
        """Modelled duration of this exchange on point-to-point links of ``gbps`` GB/s per
        direction (default LOOPBACK_LINK_GBPS): latency + largest per-peer message / rate."""
        gbps = gbps or LOOPBACK_LINK_GBPS
        if gbps <= 0 or self._world <= 1:
            return 0.0
        peer = max(max(self.send_splits, default=0), max(self.recv_splits, default=0))
        return LOOPBACK_LATENCY_US + peer * row_bytes / (gbps * 1e3)

    def _loopback(self, send: torch.Tensor, out: torch.Tensor, row_bytes: int,
                  async_op: bool):
        """No peers: receive your own send rows (the first min(sent, received) rows; any
        further received rows read as zero), optionally behind the link model."""
        m = min(self.total_send, self.total_recv)
        us = self.link_us(row_bytes) if send.is_cuda else 0.0
        if us <= 0.0:
            if m:
                out[:m].copy_(send[:m])
            if self.total_recv > m:
                out[m:].zero_()
            # the copy is stream-ordered on the current stream, which is the comm side
            # stream when called from an overlap schedule: never a no-op wait here
            return (out, _stream_done(out)) if async_op else out
        from .. import _native

        dev = send.device
        side = _side_stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        # the modelled collective is ONE kernel on the comm stream: LOOPBACK_COPY_CUS
        # workgroups move the rows, LOOPBACK_CUS of them stay resident for at least the link
        # time (the data moves while the link time runs, as on a real link; one stream, so
        # no extra hardware queue: csrc/comm/symheap.hip link_copy_kernel)
        with torch.cuda.stream(side):
            if m:
                _native.ops().link_copy(send[:m].contiguous(), out[:m], float(us),
                                        max(LOOPBACK_COPY_CUS, LOOPBACK_CUS), LOOPBACK_CUS)
            else:
                _native.ops().link_delay(float(us), int(dev.index), LOOPBACK_CUS)
            if self.total_recv > m:
                out[m:].zero_()
            ev = torch.cuda.Event()
            ev.record(side)
        # held until wait(): the allocator must not hand these blocks out again before the
        # side stream is done with them
        work = _EventWork(ev, (send, out))
        if async_op:
            return out, work
        work.wait()
        return out

    def _shmem(self, send: torch.Tensor, out: torch.Tensor, async_op: bool = False):
        """One-sided exchange: every rank puts its segment for peer p straight into p's
        symmetric receive slot at the offset where p expects rows from this rank (the
        prefix of p's receive splits), then copies its own slot out. Completion is
        stream-ordered on separate GPUs and host-ordered for ranks sharing one
        (SymmetricHeap.put_rows). The first call per (plan, row shape, dtype) is collective:
        the slot is sized for the largest receiver and the offsets are exchanged once.

        Separate GPUs (device completion) and ``async_op``: the puts, the completion
        signals / waits and the copy-out run on the device's comm side stream (every
        one-sided exchange rides it, in issue order, so the heap's epoch counters stay in
        step on all ranks) behind the current stream's work, and the returned work's
        ``wait()`` is a stream-event wait — the exchange overlaps whatever the caller
        issues next, as the RCCL path does (the reference's put was synchronous,
        DGraph/distributed/Engine.py:67-86). Returns the work object."""
        heap = shmem_heap(self.group, send.device)
        if self._shm_offsets is None:
            from ..plan.pattern import _alltoall_counts

            pre = [0]
            for n in self.recv_splits[:-1]:
                pre.append(pre[-1] + n)
            mine = torch.tensor(pre, dtype=torch.long)
            self._shm_offsets = [int(v) for v in _alltoall_counts(mine, self.group).tolist()]
        key = (tuple(send.shape[1:]), send.dtype)
        slot = self._shm_slots.get(key)
        if slot is None:
            from .symheap import _allgather_obj

            rmax = max(_allgather_obj(int(self.total_recv), self.group))
            slot = heap.alloc_tensor((max(rmax, 1),) + tuple(send.shape[1:]), send.dtype)
            self._shm_slots[key] = slot
        if async_op and heap.device_completion:
            dev = send.device
            side = _side_stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                heap.put_rows(send, slot, self.send_splits, self._shm_offsets)
                if self.total_recv:
                    out.copy_(slot[: self.total_recv])
                ev = torch.cuda.Event()
                ev.record(side)
            return _EventWork(ev, (send, out))
        heap.put_rows(send, slot, self.send_splits, self._shm_offsets)
        if self.total_recv:
            out.copy_(slot[: self.total_recv])
        # host-ordered puts, but the copy-out is enqueued on the current stream
        return _stream_done(out)


def torch_alltoallv_with_comm_map(contiguous_send_tensor: torch.Tensor,
                                  contiguous_recv_tensor: torch.Tensor,
                                  send_comm_map: torch.Tensor, recv_comm_map: torch.Tensor,
                                  rank: int, world_size: int, group=None):
    """Per-peer split exchange along dim 1 of ``[B, rows, F]`` buffers
    (alltoallv_impl.py:164-181); one all-to-all-v instead of a list-form all_to_all."""
    ss = [int(v) for v in send_comm_map.tolist()]
    rs = [int(v) for v in recv_comm_map.tolist()]
    assert len(ss) == world_size and len(rs) == world_size
    send = contiguous_send_tensor.transpose(0, 1).reshape(sum(ss), -1)
    out = AllToAllV(ss, rs, group)(send)
    contiguous_recv_tensor.copy_(out.reshape(sum(rs), contiguous_recv_tensor.shape[0],
                                             -1).transpose(0, 1))
    return list(torch.split(contiguous_recv_tensor, rs, dim=1))


def _nccl_alltoallv_with_dict(send_buffer_dict, recv_buffer_dict, rank: int, world_size: int,
                              group=None):
    """Exchange per-peer buffers keyed by peer rank (alltoallv_impl.py:134-161) with one
    all-to-all-v over their concatenation (received rows keep the sender's dtype; the
    reference forced ``.float()``)."""
    peers = range(world_size)
    ref = next(iter(send_buffer_dict.values()), None)
    if ref is None:
        ref = next(iter(recv_buffer_dict.values()))
    F = ref.shape[-1]
    ss = [send_buffer_dict[p].numel() // F if p in send_buffer_dict and p != rank else 0
          for p in peers]
    rs = [recv_buffer_dict[p].numel() // F if p in recv_buffer_dict and p != rank else 0
          for p in peers]
    send = torch.cat([send_buffer_dict[p].reshape(-1, F) for p in peers if ss[p]] or
                     [ref.new_zeros(0, F)])
    out = AllToAllV(ss, rs, group)(send)
    off = 0
    for p in peers:
        if rs[p]:
            recv_buffer_dict[p].copy_(out[off:off + rs[p]].reshape(recv_buffer_dict[p].shape))
            off += rs[p]
    return recv_buffer_dict
