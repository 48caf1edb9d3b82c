"""Whole-step HIP-graph capture for launch-bound training loops.

A training step on a small or medium graph (ogbn-arxiv / -products shapes, GraphCast's
mesh processor, the synthetic OGB-LSC runs) is hundreds of short kernels: forward,
backward, gradient sync and the optimizer. Launched one by one from Python, the host-side
launch path (~5-20 us per op through the dispatcher) is slower than the kernels themselves
and the GPU idles between them. :class:`GraphedStep` records the step once into a HIP graph
(``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and afterwards replays it with ONE launch:
the kernels keep their arguments, their stream order and their memory, so a replayed step
is the same arithmetic as an eager one (tests/test_graphed_gpu.py checks the losses match).

What the captured step must satisfy (all true for the library's models and ops):
  * static inputs: features, labels, masks and the graph stay the same tensors (their
    contents may be updated in place between replays);
  * no host synchronisation inside the step (no ``.item()``, ``nonzero``, host-side
    shape decisions from device data): the library's plan caches are built during the
    eager warmup steps and only read afterwards; native launchers only enqueue on the
    current stream;
  * the optimizer runs with ``capturable=True`` (device-side step counters); use
    :func:`make_capturable` on an existing Adam/AdamW/SGD;
  * gradients are assigned, not accumulated, inside the step (``zero_grad(set_to_none=True)``
    at its top): the captured backward then writes the same pool-owned gradient tensors on
    every replay.
Collectives (RCCL all-reduce / all-to-all with host-cached splits) are capturable as well,
so the same wrapper works under torchrun; every rank must capture the same step.

This is the launch-overhead answer the reference gets from nothing (it launches eagerly,
experiments/OGB/main.py:129-158); a tracing compiler is deliberately not used.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


def make_capturable(opt: torch.optim.Optimizer) -> torch.optim.Optimizer:
    """Switch an optimizer to device-side step counters so ``step()`` can be captured.

    Must be called before the first ``step()`` or after it: existing CPU step counters are
    moved to the parameters' device."""
    for group in opt.param_groups:
        if "capturable" not in group:
            raise ValueError(f"{type(opt).__name__} has no capturable mode")
        group["capturable"] = True
        for p in group["params"]:
            st = opt.state.get(p)
            if st and "step" in st and torch.is_tensor(st["step"]):
                st["step"] = st["step"].to(p.device, torch.float32)
    return opt


class GraphedStep:
    """Run ``step_fn()`` eagerly ``warmup`` times on a side stream, capture the next call
    into a HIP graph, then replay it on every later call.

    ``step_fn`` returns the (device) tensor to hand back, e.g. the loss; after capture the
    same static tensor is returned by every replay, updated in place. Call
    :meth:`reset` after changing anything the step reads by reference (a new graph,
    re-created parameters) to force a fresh capture.
    """

    def __init__(self, step_fn: Callable[[], Optional[torch.Tensor]], warmup: int = 3,
                 enabled: bool = True):
        self.step_fn = step_fn
        self.warmup = max(int(warmup), 1)  # >= 1 eager step: lazy plans/workspaces exist
        self.enabled = enabled and torch.cuda.is_available()
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out: Optional[torch.Tensor] = None
        self.calls = 0
        self.replays = 0

    @property
    def captured(self) -> bool:
        return self.graph is not None

    def reset(self) -> None:
        self.graph = None
        self.out = None
        self.calls = 0

    def __call__(self) -> Optional[torch.Tensor]:
        if not self.enabled:
            return self.step_fn()
        if self.graph is not None:
            self.graph.replay()
            self.replays += 1
            return self.out
        self.calls += 1
        cur = torch.cuda.current_stream()
        if self.calls <= self.warmup:
            # warmup on a side stream (what capture requires of the allocator state and of
            # the autograd engine's per-stream bookkeeping)
            side = torch.cuda.Stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                out = self.step_fn()
            cur.wait_stream(side)
            return out
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.out = self.step_fn()
        self.graph = g
        # the capture recorded the step without running it: run it once now
        g.replay()
        self.replays += 1
        return self.out
