"""Data-parallel gradient synchronisation for replicated weights (P5 / X16).

GNN weights are small (MBs) while the graph is huge, so the all-reduce is latency-bound:
one flattened fp32 bucket, one RCCL all-reduce per step (instead of DDP's per-bucket
hooks). Ring all-reduce over xGMI uses one outgoing link per step per GPU; at these sizes
that is irrelevant. ``torch.nn.parallel.DistributedDataParallel`` also works with every
model in the library; this is the lean default used by the trainers and the benchmark.
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch
import torch.distributed as dist


class GradSync:
    def __init__(self, params: Iterable[torch.nn.Parameter], group: Optional[dist.ProcessGroup] = None,
                 average: bool = False):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.group = group
        self.average = average
        self._flat: Optional[torch.Tensor] = None

    def all_reduce(self) -> None:
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        ps = [p for p in self.params]
        numel = sum(p.numel() for p in ps)
        dev = ps[0].device
        fdt = torch.float64 if any(p.dtype == torch.float64 for p in ps) else torch.float32
        if (self._flat is None or self._flat.numel() != numel or self._flat.device != dev
                or self._flat.dtype != fdt):
            self._flat = torch.empty(numel, dtype=fdt, device=dev)
        off = 0
        for p in ps:
            n = p.numel()
            if p.grad is None:
                self._flat[off:off + n].zero_()
            else:
                self._flat[off:off + n].copy_(p.grad.reshape(-1))
            off += n
        dist.all_reduce(self._flat, group=self.group)
        if self.average:
            self._flat.div_(dist.get_world_size(self.group))
        off = 0
        for p in ps:
            n = p.numel()
            v = self._flat[off:off + n].view_as(p)
            if p.grad is None:
                p.grad = v.to(p.dtype, copy=True)
            else:
                p.grad.copy_(v)
            off += n
