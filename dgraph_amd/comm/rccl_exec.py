"""Native RCCL plan executor (csrc/comm/comm_ops.cpp).

A private RCCL communicator per process group, driven with grouped ``ncclSend``/``ncclRecv``
from C++. The plan's host-cached row splits go straight to RCCL (no split tensors, no
device->host syncs), zero-size peers are skipped, several tensors (e.g. the feature rows
and their per-row scales) can share one group call, and asynchronous exchanges run on a
dedicated high-priority HIP stream whose completion event the consumer waits on — the
compute stream never blocks on the host.

Selected for :class:`~dgraph_amd.comm.alltoallv.AllToAllV` with
``DGRAPH_A2A_IMPL=native`` (default ``torch``: ProcessGroupNCCL, i.e. RCCL through
torch.distributed).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import _native


class _EventWork:
    """Completion event of an exchange on the executor's stream; the exchange's tensors are
    held until ``wait()`` (no record_stream: see comm/alltoallv.py _EventWork)."""

    def __init__(self, event: torch.cuda.Event, keep=()):
        self._ev = event
        self._keep = keep

    def wait(self):
        torch.cuda.current_stream().wait_event(self._ev)
        self._keep = ()

    def is_completed(self) -> bool:
        return self._ev.query()


class RCCLExecutor:
    _registry: Dict[int, "RCCLExecutor"] = {}

    @classmethod
    def for_group(cls, group: Optional[dist.ProcessGroup]) -> "RCCLExecutor":
        key = id(group) if group is not None else 0
        ex = cls._registry.get(key)
        if ex is None:
            ex = cls(group)
            cls._registry[key] = ex
        return ex

    def __init__(self, group: Optional[dist.ProcessGroup] = None):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.device = torch.device("cuda", torch.cuda.current_device())
        ops = _native.ops()
        uid = [ops.rccl_unique_id().numpy().tobytes() if self.rank == 0 else None]
        if self.world > 1:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(uid, src=src, group=group)
        uid_t = torch.frombuffer(bytearray(uid[0]), dtype=torch.uint8)
        self.handle = ops.rccl_comm_init(uid_t, self.world, self.rank, self.device.index)
        self.stream = torch.cuda.Stream(self.device, priority=-1)

    def alltoallv(self, sends: Sequence[torch.Tensor], recvs: Sequence[torch.Tensor],
                  send_splits: Sequence[int], recv_splits: Sequence[int],
                  async_op: bool = False):
        s = torch.tensor([int(v) for v in send_splits], dtype=torch.int64)
        r = torch.tensor([int(v) for v in recv_splits], dtype=torch.int64)
        sends = [t.contiguous() for t in sends]
        ops = _native.ops()
        if not async_op:
            ops.rccl_alltoallv(self.handle, sends, list(recvs), s, r)
            return None
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            ops.rccl_alltoallv(self.handle, sends, list(recvs), s, r)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return _EventWork(ev, tuple(sends) + tuple(recvs))

    def all_reduce(self, t: torch.Tensor) -> None:
        _native.ops().rccl_allreduce(self.handle, t)

    def close(self) -> None:
        if self.handle:
            torch.cuda.synchronize(self.device)
            _native.ops().rccl_comm_destroy(self.handle)
            self.handle = 0

    @classmethod
    def close_all(cls) -> None:
        for ex in cls._registry.values():
            ex.close()
        cls._registry.clear()
