"""Fault injection for the communication layer.

The reference has no failure handling at all: a failing rank ``exit()``s from a CUDA
macro and the survivors hang in their next collective (include/macros.hpp:18-29). Here
process groups carry timeouts and ``TORCH_NCCL_ASYNC_ERROR_HANDLING`` (comm/groups.py),
and this module lets tests provoke the failure modes on purpose, at the one place every
halo / plan exchange goes through (:class:`~dgraph_amd.comm.alltoallv.AllToAllV`).

Spec (``DGRAPH_FAULT`` environment variable or :func:`set_fault`), ``;``-separated rules
``kind[:key=value]*``:

* ``delay:ms=200[:rank=1][:every=1]``  sleep before the exchange (a straggler);
* ``corrupt[:rank=1][:call=3]``        zero the outgoing payload of that call (silent data
  corruption; plan-level checksums / loss checks must catch it);
* ``fail[:rank=1][:call=3]``           raise :class:`InjectedFault` instead of exchanging
  (a crashed rank; peers then hit the process-group timeout instead of hanging forever).

``call`` counts this process's exchanges from 1; a rule without ``rank`` applies to all.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch


class InjectedFault(RuntimeError):
    """Raised by a ``fail`` rule."""


@dataclass
class _Rule:
    kind: str
    params: Dict[str, int] = field(default_factory=dict)

    def applies(self, rank: int, call: int) -> bool:
        if "rank" in self.params and self.params["rank"] != rank:
            return False
        if "call" in self.params and self.params["call"] != call:
            return False
        every = self.params.get("every", 1)
        return every <= 1 or call % every == 0


def parse(spec: str) -> List[_Rule]:
    rules = []
    for part in filter(None, (p.strip() for p in spec.split(";"))):
        kind, *kvs = part.split(":")
        if kind not in ("delay", "corrupt", "fail"):
            raise ValueError(f"unknown fault kind {kind!r} in {spec!r}")
        params = {}
        for kv in kvs:
            k, v = kv.split("=")
            params[k.strip()] = int(v)
        rules.append(_Rule(kind, params))
    return rules


class FaultInjector:
    rules: List[_Rule] = parse(os.environ.get("DGRAPH_FAULT", ""))
    calls = 0
    log: List[str] = []

    @classmethod
    def active(cls) -> bool:
        return bool(cls.rules)

    @classmethod
    def before_exchange(cls, send: torch.Tensor, rank: int) -> torch.Tensor:
        """Apply the matching rules to one outgoing exchange; returns the payload to send."""
        cls.calls += 1
        for r in cls.rules:
            if not r.applies(rank, cls.calls):
                continue
            cls.log.append(f"{r.kind}@rank{rank}/call{cls.calls}")
            if r.kind == "delay":
                time.sleep(r.params.get("ms", 100) / 1000.0)
            elif r.kind == "corrupt":
                send = torch.zeros_like(send)
            elif r.kind == "fail":
                raise InjectedFault(f"injected failure on rank {rank}, exchange {cls.calls}")
        return send


def set_fault(spec: Optional[str]) -> None:
    """Install (or with ``None`` clear) fault rules for this process."""
    FaultInjector.rules = parse(spec or "")
    FaultInjector.calls = 0
    FaultInjector.log = []
