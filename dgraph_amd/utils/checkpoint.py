"""Checkpoint / resume (§5.4).

The reference saved only ``model_{iter}.pth`` (a DDP ``state_dict`` whose keys carry the
``module.`` prefix, GraphCast/train_graphcast.py:150-151) and had no training-state
resume. Here:

* :func:`save_checkpoint` writes ``{model, optimizer, scheduler, epoch, rng, plan_hash,
  world_size, config}`` from rank 0 (weights are replicated) atomically;
* :func:`load_checkpoint` restores it with ``weights_only=True`` (no unpickling),
  accepting both prefixed (DDP) and plain keys; a ``plan_hash`` mismatch (different
  graph / partition / world size) is reported so plans are rebuilt instead of reused;
* :func:`save_model_weights` keeps the reference's ``model_{iter}.pth`` name.
"""
from __future__ import annotations

import hashlib
import os
from typing import Optional

import torch
import torch.distributed as dist


def plan_hash(*tensors, extra: str = "") -> str:
    """Stable hash of the tensors a plan depends on (graph, partition, W, rank)."""
    h = hashlib.sha1(extra.encode())
    for t in tensors:
        t = t.detach().cpu().contiguous()
        h.update(str((tuple(t.shape), str(t.dtype))).encode())
        h.update(t.numpy().tobytes() if t.numel() < (1 << 24) else
                 t.reshape(-1)[:: max(1, t.numel() // (1 << 20))].numpy().tobytes())
    return h.hexdigest()


def _strip(sd: dict) -> dict:
    return {k[7:] if k.startswith("module.") else k: v for k, v in sd.items()}


def _rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def save_checkpoint(path: str, model, optimizer=None, scheduler=None, epoch: int = 0,
                    plan_hash_value: str = "", config: Optional[dict] = None) -> None:
    if _rank() != 0:
        return
    state = {
        "model": _strip(model.state_dict()),
        "optimizer": optimizer.state_dict() if optimizer is not None else {},
        "scheduler": scheduler.state_dict() if scheduler is not None else {},
        "epoch": int(epoch),
        "rng_cpu": torch.get_rng_state(),
        "plan_hash": plan_hash_value,
        "world_size": dist.get_world_size() if dist.is_initialized() else 1,
        "config": config or {},
    }
    if torch.cuda.is_available():
        state["rng_cuda"] = torch.cuda.get_rng_state()
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str, model, optimizer=None, scheduler=None,
                    map_location="cpu", expected_plan_hash: str = "") -> dict:
    state = torch.load(path, map_location=map_location, weights_only=True)
    target = model.module if hasattr(model, "module") else model
    target.load_state_dict(_strip(state["model"]))
    if optimizer is not None and state.get("optimizer"):
        optimizer.load_state_dict(state["optimizer"])
    if scheduler is not None and state.get("scheduler"):
        scheduler.load_state_dict(state["scheduler"])
    if "rng_cpu" in state:
        torch.set_rng_state(state["rng_cpu"])
    if "rng_cuda" in state and torch.cuda.is_available():
        torch.cuda.set_rng_state(state["rng_cuda"])
    state["plan_stale"] = bool(expected_plan_hash) and state.get("plan_hash") != expected_plan_hash
    return state


def save_model_weights(model, iteration: int, directory: str = ".") -> str:
    """``model_{iter}.pth`` = plain state_dict (reference layout; loads into DDP or not)."""
    path = os.path.join(directory, f"model_{iteration}.pth")
    if _rank() == 0:
        torch.save(model.state_dict(), path)
    return path
