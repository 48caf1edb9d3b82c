"""Shared trainer plumbing: config, resume, per-epoch metrics (§5.4-§5.6 wired together).

Every entry point (``experiments/ogb_gcn.py``, ``ogb_lsc.py``, ``graphcast.py``,
``bench.py``) builds its :class:`~dgraph_amd.utils.config.RunConfig` the same way —
defaults, then ``DGRAPH_<SECTION>_<FIELD>`` environment variables, then the CLI's own
flags, then ``--config section.field=value`` overrides — and pushes the kernel knobs into
the native library. :class:`RunSupport` then gives the training loop

* ``resume(model, opt, sched)``: restore ``{model, optimizer, scheduler, epoch, rng,
  plan_hash}`` from ``--resume`` (``weights_only`` load; a plan-hash mismatch, i.e. a
  different graph / partition / world size, is reported);
* ``end_epoch(...)``: one JSONL metrics line per epoch (``epoch_ms``, ``edges_per_s``,
  halo bytes sent per peer, comm / compute ms from the TimingReport regions, peak HBM)
  and a checkpoint every ``--checkpoint_every`` epochs.

The reference had per-run text logs and ``model_{iter}.pth`` only
(experiments/OGB/main.py:125-221, GraphCast/train_graphcast.py:150-151).
"""
from __future__ import annotations

import argparse
import os
import time
from typing import Optional, Sequence

import torch
import torch.distributed as dist

from .checkpoint import load_checkpoint, save_checkpoint
from .config import RunConfig, apply_overrides
from .metrics import ExperimentLogger, peak_memory_gb


def add_run_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    g = p.add_argument_group("run (config / resume / metrics)")
    g.add_argument("--config", action="append", default=[], metavar="SECTION.FIELD=VALUE",
                   help="RunConfig override (repeatable), applied after DGRAPH_* env vars")
    g.add_argument("--resume", default="", help="checkpoint to resume from")
    g.add_argument("--checkpoint_dir", default="", help="write checkpoints here")
    g.add_argument("--checkpoint_every", type=int, default=0,
                   help="checkpoint every N epochs (0: only at the end when a dir is set)")
    g.add_argument("--metrics_jsonl", default="",
                   help="metrics stream path (default {log_dir}/{dataset}_world{W}_metrics"
                        ".jsonl)")
    return p


def build_config(overrides: Sequence[str] = (), **explicit) -> RunConfig:
    """RunConfig from env, then explicit trainer values ``section__field=value``, then the
    ``--config`` strings."""
    cfg = RunConfig.from_env()
    for key, val in explicit.items():
        if val is None:
            continue
        sec, _, name = key.partition("__")
        setattr(getattr(cfg, sec), name, val)
    apply_overrides(cfg, list(overrides))
    return cfg


class _CommSnapshot:
    def __init__(self):
        from ..comm.alltoallv import CommStats

        self.bytes = dict(CommStats.peer_bytes_sent)
        self.calls = CommStats.calls


class RunSupport:
    def __init__(self, args, cfg: RunConfig, dataset: str, world: int, log_dir: str,
                 device: Optional[torch.device] = None, plan_hash: str = ""):
        self.args, self.cfg = args, cfg
        self.device = device
        self.plan_hash = plan_hash
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = world
        path = getattr(args, "metrics_jsonl", "") or ""
        self.logger = ExperimentLogger(os.path.dirname(path) if path else log_dir, dataset,
                                       world)
        if path:
            self.logger.jsonl = path
        self.start_epoch = 0
        self._snap = None
        self._t0 = None
        if device is not None and device.type == "cuda":
            cfg.apply()

    # -------------------------------------------------------------------------- resume
    def resume(self, model, optimizer=None, scheduler=None) -> int:
        path = getattr(self.args, "resume", "")
        if not path:
            return 0
        state = load_checkpoint(path, model, optimizer, scheduler,
                                map_location=self.device or "cpu",
                                expected_plan_hash=self.plan_hash)
        self.start_epoch = int(state.get("epoch", -1)) + 1
        if state.get("plan_stale") and self.rank == 0:
            print(f"[resume] {path}: plan hash differs (graph / partition / world size "
                  f"changed); communication plans are rebuilt", flush=True)
        if self.rank == 0:
            print(f"[resume] {path}: continuing at epoch {self.start_epoch}", flush=True)
        return self.start_epoch

    # -------------------------------------------------------------------------- epochs
    def begin_epoch(self) -> None:
        self._snap = _CommSnapshot()
        self._t0 = time.perf_counter()

    def end_epoch(self, epoch: int, model, optimizer=None, scheduler=None,
                  epoch_ms: Optional[float] = None, edges: Optional[int] = None,
                  loss: Optional[float] = None, **extra) -> dict:
        from ..comm.alltoallv import CommStats
        from .timing import TimingReport

        if epoch_ms is None:
            epoch_ms = (time.perf_counter() - self._t0) * 1e3 if self._t0 else 0.0
        per_peer = {}
        if self._snap is not None:
            for p, b in CommStats.peer_bytes_sent.items():
                d = b - self._snap.bytes.get(p, 0)
                if d:
                    per_peer[str(p)] = d
        comm_ms = None
        if TimingReport._is_initialized:
            TimingReport.resolve()
            ex = [v[-1] for k, v in TimingReport._timers.items()
                  if ("exchange" in k or "comm" in k) and v]
            comm_ms = float(sum(ex)) if ex else None
        rec = {"epoch": epoch, "epoch_ms": epoch_ms, "world_size": self.world,
               "peak_hbm_gb": round(peak_memory_gb(), 3),
               "halo_bytes_per_peer": per_peer,
               "halo_bytes_max_peer": max(per_peer.values()) if per_peer else 0}
        if edges is not None and epoch_ms > 0:
            rec["edges_per_s"] = edges / (epoch_ms / 1e3)
        if loss is not None:
            rec["loss"] = loss
        if comm_ms is not None:
            rec["comm_ms"] = comm_ms
            rec["compute_ms"] = max(epoch_ms - comm_ms, 0.0)
        rec.update(extra)
        self.logger.metrics(**rec)
        every = getattr(self.args, "checkpoint_every", 0)
        cdir = getattr(self.args, "checkpoint_dir", "")
        if cdir and every and (epoch + 1) % every == 0:
            self.checkpoint(epoch, model, optimizer, scheduler)
        return rec

    def finish(self, last_epoch: int, model, optimizer=None, scheduler=None) -> None:
        if getattr(self.args, "checkpoint_dir", "") and last_epoch >= 0:
            self.checkpoint(last_epoch, model, optimizer, scheduler)

    def checkpoint(self, epoch: int, model, optimizer=None, scheduler=None) -> str:
        path = os.path.join(self.args.checkpoint_dir, f"checkpoint_epoch{epoch}.pt")
        save_checkpoint(path, model, optimizer, scheduler, epoch, self.plan_hash,
                        self.cfg.to_dict())
        latest = os.path.join(self.args.checkpoint_dir, "checkpoint_latest.pt")
        save_checkpoint(latest, model, optimizer, scheduler, epoch, self.plan_hash,
                        self.cfg.to_dict())
        return path
