"""Communicator and backend-engine contracts.

Keeps the public contract of the reference's ``CommunicatorBase``
(DGraph/CommunicatorBase.py:17-50) and ``BackendEngine`` (DGraph/distributed/Engine.py:18-106)
so user code written against DGraph keeps working; the implementations are new.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional, Tuple

import torch


class CommunicatorBase(ABC):
    _is_initialized: bool = False

    def __init__(self):
        self.backend = ""

    @abstractmethod
    def init_process_group(self, backend: str, **kwargs):
        raise NotImplementedError

    @abstractmethod
    def get_rank(self) -> int:
        raise NotImplementedError

    @abstractmethod
    def get_world_size(self) -> int:
        raise NotImplementedError

    @abstractmethod
    def barrier(self) -> None:
        raise NotImplementedError

    @abstractmethod
    def scatter(self, *args, **kwargs):
        raise NotImplementedError

    @abstractmethod
    def gather(self, *args, **kwargs):
        raise NotImplementedError

    @abstractmethod
    def destroy(self) -> None:
        raise NotImplementedError


class BackendEngine:
    """Engine contract used by :class:`~dgraph_amd.comm.communicator.Communicator`.

    ``put`` is synchronous from the caller's point of view (stream-ordered on GPU: the
    receive buffer is valid for any kernel later enqueued on the current stream).
    Two-sided engines ignore ``remote_offsets``; one-sided engines write rank ``i``'s
    segment at ``remote_offsets[i]`` of rank ``i``'s receive buffer (Engine.py:67-86).
    """

    def init_process_group(self, *args, **kwargs):
        raise NotImplementedError

    def get_rank(self) -> int:
        raise NotImplementedError

    def get_world_size(self) -> int:
        raise NotImplementedError

    def scatter(self, *args, **kwargs) -> torch.Tensor:
        raise NotImplementedError

    def gather(self, *args, **kwargs) -> torch.Tensor:
        raise NotImplementedError

    def put(
        self,
        send_buffer: torch.Tensor,
        recv_buffer: torch.Tensor,
        send_offsets: torch.Tensor,
        recv_offsets: torch.Tensor,
        remote_offsets: Optional[torch.Tensor] = None,
    ) -> None:
        raise NotImplementedError

    def allocate_buffer(
        self, size: Tuple[int, ...], dtype: torch.dtype, device: torch.device
    ) -> torch.Tensor:
        return torch.empty(size, dtype=dtype, device=device)

    def finalize(self) -> None:
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError
