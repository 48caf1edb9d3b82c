"""GraphCast training (experiments/GraphCast/train_graphcast.py behaviour).

Graph x data hybrid parallelism: ``procs_per_graph`` ranks share one partitioned
GraphCast graph (latitude bands; halo exchanges inside the graph group), and the
``W / procs_per_graph`` graph groups train on different samples (replica sampler); the
replicated weights are averaged over all ranks with one flat all-reduce.

Schedule: linear warm-up (``num_iters_step1``), cosine decay (``num_iters_step2``) and a
constant fine-tuning rate ``lr_step3`` — stepped once per iteration (the reference stepped
twice and used ``num_iters_step3 / lr`` as the fine-tuning factor). Gradient clipping at
``grad_clip_norm``; checkpoints ``model_{iter}.pth`` every ``save_freq`` iterations when a
``checkpoint_dir`` is given. Loss: mean squared error over every grid point and channel
of the whole graph (global mean over the graph group).

CLI: ``python -m dgraph_amd.experiments.graphcast --backend nccl --iters 10``.
"""
from __future__ import annotations

import argparse
import math
import os
import time
from typing import Optional

import torch
import torch.distributed as dist

from .. import Communicator
from ..data.graphcast_graph import (build_global_graph, load_mesh_placement,
                                   partition_graphcast_graph)
from ..data.weather import SyntheticWeatherDataset
from ..models.graphcast import Config, DGraphCast
from ..ops.dense import deferred_wgrad
from ..parallel.grad_sync import GradSync
from ..utils.master_weights import MasterWeights
from ..utils.metrics import print_on_rank_zero
from ..utils.timing import TimingReport
from ..utils.trainer import RunSupport, add_run_args, build_config


def make_scheduler(optimizer, tc):
    s1, s2 = tc.num_iters_step1, tc.num_iters_step2

    def factor(it: int) -> float:
        if it < s1:
            return 1e-3 + (1.0 - 1e-3) * it / max(s1, 1)
        if it < s1 + s2:
            return 0.5 * (1.0 + math.cos(math.pi * (it - s1) / max(s2, 1)))
        return tc.lr_step3 / tc.lr

    return torch.optim.lr_scheduler.LambdaLR(optimizer, factor)


def _device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class GraphCastTrainer:
    def __init__(self, comm, cfg: Optional[Config] = None, dtype: torch.dtype = torch.float32,
                 checkpoint_dir: Optional[str] = None, global_graph=None, support=None,
                 mesh_vertex_placement: Optional[str] = None):
        self.comm = comm
        self.cfg = cfg or Config()
        self.device = _device()
        self.dtype = dtype
        self.checkpoint_dir = checkpoint_dir
        m = self.cfg.model
        g = global_graph or build_global_graph(m.mesh_level, tuple(self.cfg.data.latlon_res))
        self.prank, self.psize = comm.partition_rank(), comm.partition_size()
        part = comm.partition
        self.replica, self.num_replicas = ((part.partition_id, comm.get_world_size() // part.ranks_per_graph)
                                           if part is not None else (0, 1))
        mesh_part = None
        if mesh_vertex_placement:
            # the reference's mesh_vertex_rank_placement.pt (GraphCast/dataset.py:244); the
            # grid placement follows it by the reference's rule: each grid vertex on the
            # rank of its grid2mesh mesh destination (graphcast_graph.grid_placement_from_g2m)
            mesh_part = load_mesh_placement(mesh_vertex_placement, g.mesh_xyz.shape[0],
                                            self.psize)
        self.graph = partition_graphcast_graph(g, self.prank, self.psize, mesh_part=mesh_part,
                                               group=comm.group).to(self.device)
        self.dataset = SyntheticWeatherDataset(self.graph, self.cfg.data.num_channels_climate,
                                               self.cfg.data.num_samples_per_year_train)
        torch.manual_seed(0)
        self.model = DGraphCast(self.cfg, comm).to(self.device, dtype)
        self.sync = GradSync(self.model.parameters())
        lr = self.cfg.training.lr
        self.masters = None
        if dtype != torch.float32:
            # bf16 compute, fp32 master weights + optimizer state (utils/master_weights.py)
            self.masters = MasterWeights(self.model, lambda ps: torch.optim.Adam(ps, lr=lr))
            self.optimizer = self.masters.optimizer
        else:
            self.optimizer = torch.optim.Adam(self.model.parameters(), lr=lr)
        self.scheduler = make_scheduler(self.optimizer, self.cfg.training)
        self.support = support
        n = torch.tensor([float(self.graph.num_local_grid * self.cfg.model.output_grid_dim)],
                         device=self.device)
        if self.psize > 1:
            dist.all_reduce(n, group=comm.group)
        self.n_global = float(n)
        self.iter = 0
        self.history = []

    def sample(self, step: int):
        idx = (step * self.num_replicas + self.replica) % len(self.dataset)
        x, y = self.dataset[idx]
        return x.to(self.device, self.dtype), y.to(self.device, self.dtype)

    def step(self, x, y) -> float:
        self.model.train()
        self.optimizer.zero_grad(set_to_none=True)
        out = self.model(x, self.graph)
        loss = ((out.float() - y.float()) ** 2).sum() / self.n_global
        with deferred_wgrad():  # weight gradients off the backward's critical path
            loss.backward()
        # sum over the graph group = this replica's gradient; mean over replicas
        self.sync.all_reduce()
        if self.num_replicas > 1:
            for p in self.model.parameters():
                if p.grad is not None:
                    p.grad.div_(self.num_replicas)
        torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.cfg.training.grad_clip_norm)
        if self.masters is not None:
            self.masters.step()
        else:
            self.optimizer.step()
        self.scheduler.step()
        self.iter += 1
        lv = loss.detach()
        if self.psize > 1:
            dist.all_reduce(lv, group=self.comm.group)
        return float(lv)

    def _ckpt_model(self):
        return self.masters if self.masters is not None else self.model

    def train(self, iters: int) -> float:
        last = float("nan")
        sup = self.support
        if sup is not None:
            self.iter = sup.resume(self._ckpt_model(), self.optimizer, self.scheduler)
        while self.iter < iters:
            x, y = self.sample(self.iter)
            if sup is not None:
                sup.begin_epoch()
            t0 = time.perf_counter()
            last = self.step(x, y)
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            self.history.append({"iter": self.iter, "loss": last, "ms": ms})
            print_on_rank_zero(f"iter {self.iter:5d} | loss {last:.5f} | {ms:.1f} ms")
            if sup is not None:  # one metrics record / checkpoint slot per iteration
                sup.end_epoch(self.iter - 1, self._ckpt_model(), self.optimizer,
                              self.scheduler, epoch_ms=ms, loss=last)
            if (self.checkpoint_dir and self.iter % self.cfg.training.save_freq == 0
                    and self.comm.get_rank() == 0):
                os.makedirs(self.checkpoint_dir, exist_ok=True)
                torch.save(self.model.state_dict(),
                           os.path.join(self.checkpoint_dir, f"model_{self.iter}.pth"))
        if sup is not None:
            sup.finish(self.iter - 1, self._ckpt_model(), self.optimizer, self.scheduler)
        return last


def main(backend: str = "nccl", procs_per_graph: int = -1, iters: int = 10,
         mesh_level: int = 6, grid: str = "721x1440", hidden_dim: int = 128,
         processor_layers: int = 4, channels: int = 73, dtype: str = "fp32",
         checkpoint_dir: Optional[str] = None, test_run: bool = False, run_args=None,
         log_dir: str = "logs", mesh_vertex_placement: Optional[str] = None):
    rcfg = build_config(getattr(run_args, "config", ()), comm__backend=backend,
                        comm__ranks_per_graph=procs_per_graph, model__name="graphcast",
                        model__hidden=hidden_dim, model__num_layers=processor_layers,
                        model__dtype=dtype, train__epochs=iters, train__log_dir=log_dir,
                        data__dataset=f"graphcast-{grid}-level{mesh_level}")
    cfg = Config()
    cfg.model.mesh_level = mesh_level
    cfg.model.hidden_dim = hidden_dim
    cfg.model.processor_layers = processor_layers
    cfg.model.input_grid_dim = cfg.model.output_grid_dim = channels
    cfg.data.num_channels_climate = channels
    cfg.data.latlon_res = tuple(int(v) for v in grid.split("x"))
    comm = Communicator.init_process_group(backend, ranks_per_graph=procs_per_graph)
    if not TimingReport._is_initialized:
        TimingReport.init(comm)
    support = None
    if run_args is not None:
        support = RunSupport(run_args, rcfg, rcfg.data.dataset, comm.get_world_size(),
                             log_dir, _device())
    tr = GraphCastTrainer(comm, cfg, torch.bfloat16 if dtype == "bf16" else torch.float32,
                          checkpoint_dir, support=support,
                          mesh_vertex_placement=mesh_vertex_placement)
    last = tr.train(1 if test_run else iters)
    return tr, last


def cli(argv=None):
    p = argparse.ArgumentParser(description="GraphCast training on synthetic weather data")
    p.add_argument("--backend", default="nccl")
    p.add_argument("--procs_per_graph", type=int, default=-1)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--mesh_level", type=int, default=6)
    p.add_argument("--grid", default="721x1440")
    p.add_argument("--hidden_dim", type=int, default=128)
    p.add_argument("--processor_layers", type=int, default=4)
    p.add_argument("--channels", type=int, default=73)
    p.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--test_run", action="store_true")
    p.add_argument("--log_dir", default="logs")
    p.add_argument("--mesh_vertex_placement", default=None,
                   help="mesh_vertex_rank_placement.pt: int tensor [V_mesh] of ranks (the "
                        "reference's placement file; grid vertices follow their mesh source)")
    add_run_args(p)  # --checkpoint_dir: model_{iter}.pth (reference layout) + resumable state
    a = p.parse_args(argv)
    run_keys = ("config", "resume", "checkpoint_every", "metrics_jsonl", "checkpoint_dir")
    kw = {k: v for k, v in vars(a).items() if k not in run_keys}
    main(**kw, checkpoint_dir=a.checkpoint_dir or None, run_args=a)
    Communicator.instance().destroy()


if __name__ == "__main__":
    cli()
