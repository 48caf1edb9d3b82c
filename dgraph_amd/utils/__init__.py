"""Timers, logging, configuration, checkpointing."""
from .data_splitting import largest_split, split_per_rank
from .timing import TimingReport

__all__ = ["TimingReport", "largest_split", "split_per_rank"]


def try_barrier(group=None) -> None:
    """Barrier that tolerates an uninitialised process group (DGraph/utils.py:30-34 only
    swallowed every exception, hiding real failures)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier(group=group)


def check_dist_initialized() -> None:
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        raise RuntimeError("torch.distributed is not initialized")


def check_nccl_availability() -> None:
    """RCCL is torch's ``nccl`` backend on ROCm."""
    import torch.distributed as dist

    if not dist.is_nccl_available():
        raise RuntimeError("RCCL (torch 'nccl' backend) is not available")
