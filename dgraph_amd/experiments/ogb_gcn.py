"""OGB GCN trainer (experiments/OGB/main.py:50-358 behaviour).

Full-graph training of :class:`~dgraph_amd.models.gcn.CommAwareGCN` on a vertex-partitioned
OGB node-property graph: per epoch a barrier, event-timed forward / backward / Adam step,
cross-entropy on the training vertices, validation from the same forward, then a final
test pass. Logs use the reference's file names (``{log_dir}/{dataset}_world{W}_run{r}_*.log``,
``{dataset}_timing_report_world{W}.json``, loss/accuracy plots); gradients of the
replicated weights are synchronised with one flat RCCL all-reduce (:class:`GradSync`)
instead of DDP. Differences: ``dataset`` also accepts ``papers100M`` / ``proteins``
(synthetic when ogb is absent), the placement file is loaded with ``weights_only=True``,
and ``dtype="bf16"`` runs the layers in bfloat16 autocast.

CLI: ``python -m dgraph_amd.experiments.ogb_gcn --backend nccl --dataset arxiv``
(or ``examples/ogb/main.py``), under torchrun for W > 1.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F

from .. import Communicator
from ..data.ogb_comm import DGraphOGBDataset
from ..models.gcn import CommAwareGCN
from ..parallel.grad_sync import GradSync
from ..parallel.halo import HaloExchange
from ..utils.metrics import (calculate_accuracy, dist_print_ephemeral, make_experiment_log,
                             write_experiment_log)
from ..utils.timing import TimingReport, region
from ..utils.trainer import RunSupport, add_run_args, build_config

NUM_CLASSES = {"arxiv": 40, "products": 47, "papers100M": 172, "proteins": 112}


def _device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def visualize_trajectories(traj: np.ndarray, title: str, path: str, rank: int = 0) -> None:
    """Mean +- std over runs (experiments/OGB/utils.py:45-58); skipped without matplotlib."""
    if rank != 0:
        return
    np.save(path.rsplit(".", 1)[0] + ".npy", traj)
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:  # pragma: no cover - optional dependency
        return
    mean, std = traj.mean(0), traj.std(0)
    x = np.arange(traj.shape[1])
    fig, ax = plt.subplots(figsize=(6, 4))
    ax.plot(x, mean)
    ax.fill_between(x, mean - std, mean + std, alpha=0.3)
    ax.set_title(title)
    ax.set_xlabel("epoch")
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)


def run_experiment(dataset: DGraphOGBDataset, comm, lr: float, epochs: int, log_prefix: str,
                   hidden_dims: int = 256, num_classes: int = 40, device=None,
                   dtype: str = "fp32", seed: int = 0, support: Optional[RunSupport] = None,
                   cuda_graph: bool = False):
    device = device or _device()
    rank = comm.get_rank()
    x, y, cp = dataset[0]
    x, y = x.to(device), y.to(device)
    cp = cp.to(device) if hasattr(cp, "to") else cp
    masks = {k: v.to(device) for k, v in dataset.get_masks().items()}
    torch.manual_seed(seed)
    world = comm.get_world_size()
    model = CommAwareGCN(x.shape[1], hidden_dims, num_classes,
                         HaloExchange(comm) if world > 1 else None, comm).to(device)
    sync = GradSync(model.parameters(), group=comm.group)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    amp = dtype == "bf16"
    graphed = None
    if cuda_graph and device.type == "cuda":
        # whole-step HIP graph: one launch per epoch instead of hundreds (the arxiv-shaped
        # step is launch-bound); the TimingReport regions are not recorded in this mode
        from dgraph_amd.utils.graphed import GraphedStep, make_capturable

        make_capturable(opt)

    def fwd():
        with torch.autocast(device.type, dtype=torch.bfloat16, enabled=amp):
            return model(x, cp).float()

    tl, vl, va, times = [], [], [], []
    for k in ("training_loss", "validation_loss", "validation_accuracy"):
        make_experiment_log(f"{log_prefix}_{k}.log", rank)
    n_train = torch.tensor([float(masks["train_mask"].sum())], device=device)
    if world > 1:
        torch.distributed.all_reduce(n_train, group=comm.group)
    # message edges per epoch (2 propagation layers over every rank's local edge list)
    le = getattr(cp, "local_edge_list", None)
    n_edges = torch.tensor([float(le.shape[0]) if le is not None else 0.0], device=device)
    if world > 1:
        torch.distributed.all_reduce(n_edges, group=comm.group)
    edges_per_epoch = 2 * int(n_edges.item())
    tm = masks["train_mask"]

    def train_step():
        opt.zero_grad(set_to_none=True)
        out = fwd()
        # global mean over all ranks' training vertices (the reference averaged per rank)
        loss = F.cross_entropy(out[tm], y[tm].reshape(-1), reduction="sum") / n_train
        loss.backward()
        sync.all_reduce()
        opt.step()
        return loss, out

    if cuda_graph and device.type == "cuda":
        # masked indexing syncs on the mask's count: capture with precomputed indices
        ti = torch.nonzero(tm.reshape(-1)).reshape(-1)
        yt = y[ti].reshape(-1)

        def train_step():  # noqa: F811
            opt.zero_grad(set_to_none=True)
            out = fwd()
            loss = F.cross_entropy(out.index_select(0, ti), yt, reduction="sum") / n_train
            loss.backward()
            sync.all_reduce()
            opt.step()
            return loss, out

        graphed = GraphedStep(train_step, warmup=1)
    start = support.resume(model, opt) if support is not None else 0
    epoch = start - 1
    nan = float("nan")  # resumed runs: the epochs before the checkpoint are not re-logged
    tl, vl, va = [nan] * start, [nan] * start, [nan] * start
    for epoch in range(start, epochs):
        model.train()
        comm.barrier()
        _sync(device)
        if support is not None:
            support.begin_epoch()
        t0 = time.perf_counter()
        if graphed is not None:
            loss, out = graphed()
        else:
            opt.zero_grad(set_to_none=True)
            with region("forward"):
                out = fwd()
            # global mean over all ranks' training vertices (the reference averaged per rank)
            loss = F.cross_entropy(out[tm], y[tm].reshape(-1), reduction="sum") / n_train
            with region("backward"):
                loss.backward()
            sync.all_reduce()
            opt.step()
        comm.barrier()
        _sync(device)
        ms = (time.perf_counter() - t0) * 1e3
        lt = loss.detach().clone()
        if world > 1:
            torch.distributed.all_reduce(lt, group=comm.group)
        times.append(ms)
        tl.append(float(lt))
        dist_print_ephemeral(f"Epoch {epoch:4d} | loss: {float(lt):.4f} | {ms:.1f} ms", rank)
        write_experiment_log(str(float(lt)), f"{log_prefix}_training_loss.log", rank)
        with torch.no_grad():
            vm = masks["val_mask"]
            vo = out[vm].detach()
            vloss = F.cross_entropy(vo, y[vm].reshape(-1)) if vo.numel() else torch.zeros(())
            vacc = calculate_accuracy(torch.log_softmax(vo, 1), y[vm]) * 100.0
        vl.append(float(vloss))
        va.append(vacc)
        write_experiment_log(str(float(vloss)), f"{log_prefix}_validation_loss.log", rank)
        write_experiment_log(f"Validation Accuracy: {vacc:.2f}",
                             f"{log_prefix}_validation_accuracy.log", rank)
        if support is not None:
            support.end_epoch(epoch, model, opt, epoch_ms=ms, edges=edges_per_epoch,
                              loss=float(lt), val_loss=float(vloss), val_acc=vacc)
    if support is not None:
        support.finish(epoch, model, opt)
    model.eval()
    with torch.no_grad():
        out = fwd()
        sm = masks["test_mask"]
        to = out[sm]
        tloss = F.cross_entropy(to, y[sm].reshape(-1)) if to.numel() else torch.zeros(())
        tacc = calculate_accuracy(torch.log_softmax(to, 1), y[sm]) * 100.0
    test_log = f"{log_prefix}_test_results.log"
    make_experiment_log(test_log, rank)
    write_experiment_log("loss,accuracy", test_log, rank)
    write_experiment_log(f"{float(tloss)},{tacc}", test_log, rank)
    make_experiment_log(f"{log_prefix}_training_times.log", rank)
    for t in times:
        write_experiment_log(str(t), f"{log_prefix}_training_times.log", rank)
    avg = float(np.mean(times[1:])) if len(times) > 1 else float(times[0]) if times else 0.0
    make_experiment_log(f"{log_prefix}_runtime_experiment.log", rank)
    write_experiment_log(f"Average time per epoch (excl. first): {avg:.4f} ms",
                         f"{log_prefix}_runtime_experiment.log", rank)
    if rank == 0:
        print(f"\nTest  | loss: {float(tloss):.4f} | accuracy: {tacc:.2f}%", flush=True)
    return np.array(tl), np.array(vl), np.array(va)


def main(backend: str = "nccl", dataset: str = "arxiv", epochs: int = 10, lr: float = 1e-3,
         runs: int = 1, hidden_dims: int = 256, log_dir: str = "logs",
         node_rank_placement_file: Optional[str] = None, root_dir: Optional[str] = None,
         dtype: str = "fp32", synthetic_scale: float = 1.0, cuda_graph: bool = False,
         run_args=None):
    if dataset not in NUM_CLASSES:
        raise ValueError(f"Unsupported dataset '{dataset}'. Choose from {list(NUM_CLASSES)}")
    cfg = build_config(getattr(run_args, "config", ()), comm__backend=backend,
                       model__name="gcn", model__hidden=hidden_dims, model__dtype=dtype,
                       train__epochs=epochs, train__lr=lr, train__log_dir=log_dir,
                       data__dataset=dataset, data__scale=synthetic_scale)
    comm = Communicator.init_process_group(cfg.comm.backend.lower())
    rank, world = comm.get_rank(), comm.get_world_size()
    device = _device()
    if not TimingReport._is_initialized:
        TimingReport.init(comm)
    if rank == 0:
        os.makedirs(log_dir, exist_ok=True)
    placement = None
    if node_rank_placement_file is not None:
        placement = torch.load(node_rank_placement_file, weights_only=True)
    ds = DGraphOGBDataset(f"ogbn-{dataset}", comm, node_rank_placement=placement,
                          root_dir=root_dir, synthetic_scale=synthetic_scale)
    tr = np.zeros((runs, epochs))
    vl = np.zeros((runs, epochs))
    va = np.zeros((runs, epochs))
    support = None
    if run_args is not None:
        support = RunSupport(run_args, cfg, dataset, world, log_dir, device)
    for run in range(runs):
        prefix = f"{log_dir}/{dataset}_world{world}_run{run}"
        tr[run], vl[run], va[run] = run_experiment(
            ds, comm, lr, epochs, prefix, hidden_dims, NUM_CLASSES[dataset], device, dtype,
            seed=run, support=support if run == 0 else None, cuda_graph=cuda_graph)
    TimingReport.resolve()
    if rank == 0:
        TimingReport.dump(f"{log_dir}/{dataset}_timing_report_world{world}.json")
    visualize_trajectories(tr, "Training Loss", f"{log_dir}/training_loss.png", rank)
    visualize_trajectories(vl, "Validation Loss", f"{log_dir}/validation_loss.png", rank)
    visualize_trajectories(va, "Validation Accuracy", f"{log_dir}/validation_accuracy.png",
                           rank)
    return tr, vl, va


def cli(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--backend", default="nccl")
    p.add_argument("--dataset", default="arxiv")
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--runs", type=int, default=1)
    p.add_argument("--hidden_dims", type=int, default=256)
    p.add_argument("--log_dir", default="logs")
    p.add_argument("--node_rank_placement_file", default=None)
    p.add_argument("--root_dir", default=None)
    p.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--synthetic_scale", type=float, default=1.0)
    p.add_argument("--cuda_graph", action="store_true",
                   help="capture the training step into a HIP graph and replay it")
    add_run_args(p)
    a = p.parse_args(argv)
    run_keys = ("config", "resume", "checkpoint_dir", "checkpoint_every", "metrics_jsonl")
    kw = {k: v for k, v in vars(a).items() if k not in run_keys}
    main(**kw, run_args=a)
    Communicator.instance().destroy()


if __name__ == "__main__":
    cli()
