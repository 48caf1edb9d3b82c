"""Timers, logging, configuration, checkpointing."""
from .data_splitting import largest_split, split_per_rank
from .timing import TimingReport

__all__ = ["TimingReport", "largest_split", "split_per_rank"]
