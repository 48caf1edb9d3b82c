"""Experiment logging: the reference's rank-0 log files plus a JSONL metrics stream.

Reference layout (experiments/OGB/utils.py:12-29, OGB/main.py:125-221):
``{log_dir}/{dataset}_world{W}_run{run}_{training_loss|validation_loss|
validation_accuracy|test_results|training_times|runtime_experiment}.log``.
Added: one JSON object per epoch in ``{log_dir}/{dataset}_world{W}_metrics.jsonl`` with
``epoch_ms``, ``edges_per_s``, halo bytes, peak HBM (§5.5 "MI355X equivalent").
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Optional

import torch
import torch.distributed as dist


def _rank0() -> bool:
    return not dist.is_initialized() or dist.get_rank() == 0


def make_experiment_log(fname: str, rank: int = 0) -> None:
    if rank == 0:
        os.makedirs(os.path.dirname(fname) or ".", exist_ok=True)
        open(fname, "w").close()


def write_experiment_log(msg: str, fname: str, rank: int = 0) -> None:
    if rank == 0:
        with open(fname, "a") as f:
            f.write(str(msg) + "\n")


def dist_print_ephemeral(msg: str, rank: int = 0) -> None:
    if rank == 0:
        print(msg, end="\r", flush=True)


def print_on_rank_zero(*a, **kw) -> None:
    if _rank0():
        print(*a, **kw, flush=True)


def calculate_accuracy(pred: torch.Tensor, labels: torch.Tensor) -> float:
    if pred.numel() == 0:
        return 0.0
    return float((pred.argmax(-1) == labels).float().mean())


class ExperimentLogger:
    """Writes the reference's per-run log files and a JSONL metrics stream (rank 0)."""

    def __init__(self, log_dir: str, dataset: str, world_size: int, run: int = 0):
        self.prefix = os.path.join(log_dir, f"{dataset}_world{world_size}_run{run}")
        self.jsonl = os.path.join(log_dir, f"{dataset}_world{world_size}_metrics.jsonl")
        self.rank0 = _rank0()
        if self.rank0:
            os.makedirs(log_dir, exist_ok=True)
            for k in ("training_loss", "validation_loss", "validation_accuracy",
                      "test_results", "training_times", "runtime_experiment"):
                make_experiment_log(f"{self.prefix}_{k}.log")

    def log(self, kind: str, value) -> None:
        if self.rank0:
            write_experiment_log(value, f"{self.prefix}_{kind}.log")

    def metrics(self, **fields) -> None:
        if self.rank0:
            fields.setdefault("time", time.time())
            with open(self.jsonl, "a") as f:
                f.write(json.dumps(fields) + "\n")


def peak_memory_gb(device: Optional[torch.device] = None) -> float:
    if torch.cuda.is_available():
        return torch.cuda.max_memory_allocated(device) / 1e9
    return 0.0
