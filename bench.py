#!/usr/bin/env python3
"""Headline benchmark: full-graph GraphSAGE training on an ogbn-papers100M-shaped graph.

BASELINE.json metric: "edges/sec + epoch time, ogbn-papers100M 3-layer GraphSAGE at
1/2/4/8 MI355X". One process per GPU (torchrun), vertex-partitioned graph (contiguous
partition of a synthetic graph with the papers100M shape: 111,059,956 nodes,
1,615,685,872 directed edges symmetrised to ~3.23B messages per layer, 128 features,
172 classes), RCCL all-to-all-v halo exchange overlapped with interior aggregation.

A step = forward over ALL vertices (3 SAGE-mean layers, hidden 256, bf16 compute, fp32
master weights) + masked cross-entropy on the train split + backward + gradient
all-reduce + Adam step (the reference's epoch, experiments/OGB/main.py:129-158).

    edges_per_s = num_layers * E_msg / epoch_s     (E_msg = symmetrised message edges)

The whole graph is fixed as N grows (strong scaling). Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# large, long-lived activations + transient SpMM buffers: avoid allocator fragmentation
# (expandable segments are unsupported on ROCm; forbid splitting huge cached blocks so a
#  freed 57 GB activation block is never carved up by a 38 GB request)
os.environ.setdefault("PYTORCH_ALLOC_CONF", "max_split_size_mb:512")

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--shape", default="ogbn-papers100M")
    ap.add_argument("--scale", type=float, default=1.0, help="shape scale (debug only)")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--global-frac", type=float, default=0.05)
    ap.add_argument("--window", type=int, default=1 << 14)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--rehearse-world", type=int, default=0,
                    help="single process: run rank --rehearse-rank of a W-way partition with "
                         "a loopback halo exchange (per-rank compute + memory; no peers)")
    ap.add_argument("--rehearse-rank", type=int, default=0)
    ap.add_argument("--profile-ops", default="",
                    help="after the timed steps, profile one extra step with "
                         "torch.profiler and write the per-op device-time table here")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def _profile_one_step(step, path):
    """Per-aten-op device time of one (untimed) step, grouped by input shape."""
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    with open(path, "w") as f:
        f.write(ka.table(sort_by="self_cuda_time_total", row_limit=60, max_name_column_width=60,
                         max_shapes_column_width=90))


def main():
    args = parse()
    from dgraph_amd import Communicator
    from dgraph_amd.data.synthetic import SHAPES, build_partition, node_data
    from dgraph_amd.models.sage import GraphSAGE
    from dgraph_amd.parallel.dist_graph import DistGraph
    from dgraph_amd.parallel.grad_sync import GradSync

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    comm = Communicator.init_process_group("nccl")
    rank, world = comm.get_rank(), comm.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")
    shape = SHAPES[args.shape]
    if args.scale != 1.0:
        shape = shape.scaled(args.scale)

    t0 = time.time()
    rehearse = args.rehearse_world > 1 and world == 1
    p_rank, p_world = (args.rehearse_rank, args.rehearse_world) if rehearse else (rank, world)
    part = build_partition(shape, p_rank, p_world, dev, seed=args.seed,
                           global_frac=args.global_frac, window=args.window, rehearse=rehearse)
    csr = part["csr"]
    if p_world == 1:
        csr.num_cols = part["L"]
    graph = DistGraph(csr, part["L"], part["H"], part["send_local_idx"], part["send_splits"],
                      # the synthetic graph is symmetrised, so the interior (local x local)
                      # block is symmetric at every W: its transpose is never materialised
                      part["recv_splits"], comm.group, symmetric=True,
                      overlap=not args.no_overlap)
    graph.prepare_backward()
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    x, y, train = node_data(shape, p_rank, part["offsets"], dev, seed=args.seed, dtype=dtype)
    train_idx = torch.nonzero(train, as_tuple=True)[0]
    y_train = y[train_idx]
    del y, train
    e_local = torch.tensor([graph.interior.nnz + (graph.halo.nnz if graph.halo else 0),
                            train_idx.numel(), part["H"]], dtype=torch.long, device=dev)
    if world > 1:
        dist.all_reduce(e_local)
    E_msg, n_train, halo_total = (int(v) for v in e_local.tolist())
    log(rank, f"graph built in {time.time() - t0:.1f}s: V={shape.num_nodes} E_msg={E_msg} "
              f"halo_rows_total={halo_total} train={n_train}")

    torch.manual_seed(args.seed)
    model = GraphSAGE(shape.num_features, args.hidden, shape.num_classes, args.layers).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr,
                           fused=dev.type == "cuda")
    sync = GradSync(model.parameters(), group=None) if world > 1 else None
    inv_n = 1.0 / max(n_train, 1)

    def step():
        # all-vertex forward; logits of the train split leave the fused stack
        logits = model(x, graph, out_rows=train_idx).float()
        loss = torch.nn.functional.cross_entropy(logits, y_train, reduction="sum") * inv_n
        loss.backward()
        if sync is not None:
            sync.all_reduce()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    def barrier_sync():
        if world > 1:
            dist.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for i in range(args.warmup):
        l = step()
        if args.verbose:
            log(rank, f"warmup {i} loss {float(l.detach()):.4f}")
    barrier_sync()
    if dev.type == "cuda":
        torch.cuda.reset_peak_memory_stats()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        l = step()
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    if args.profile_ops and rank == 0:
        _profile_one_step(step, args.profile_ops)
    ms = torch.tensor([elapsed * 1000.0 / max(args.steps, 1)], dtype=torch.float64,
                      device=dev)
    if world > 1:
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    ms_per_step = float(ms.item())
    lt = l.detach().reshape(1).double()
    if world > 1:
        dist.all_reduce(lt)  # each rank holds its share of the global mean loss
    final_loss = float(lt.item())
    peak_gb = torch.cuda.max_memory_allocated() / 1e9 if dev.type == "cuda" else 0.0
    edges_per_s = args.layers * E_msg / (ms_per_step / 1000.0)
    if rehearse:
        # not a whole-job number: one rank's compute with a loopback exchange
        print(json.dumps({"rehearsal": True, "rank": p_rank, "world": p_world,
                          "ms_per_step_compute_loopback": ms_per_step, "L": part["L"],
                          "H": part["H"], "E_local": E_msg, "peak_mem_gb": round(peak_gb, 2),
                          "final_loss_local": final_loss}), flush=True)
    elif rank == 0:
        rec = {
            "metric": "edges_per_s",
            "value": edges_per_s,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "epoch_ms": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": (f"synthetic {shape.name}-shaped graph (V={shape.num_nodes}, "
                     f"directed={shape.num_directed_edges}, symmetrised E_msg={E_msg}, "
                     f"global_frac={args.global_frac}, window={args.window}), random "
                     f"features/labels, random-init weights"),
            "config": {
                "model": f"GraphSAGE-mean {args.layers}-layer hidden {args.hidden}",
                "global_batch": shape.num_nodes,
                "seq_len": None,
                "parallelism": f"graph-partition{world} (RCCL all-to-all-v halo) + dp-allreduce",
                "dataset_shape": shape.name,
                "num_layers": args.layers,
                "hidden": args.hidden,
                "E_msg": E_msg,
                "halo_rows_total": halo_total,
                "train_nodes": n_train,
            },
            "final_loss": final_loss,
            "peak_mem_gb_rank0": round(peak_gb, 2),
        }
        print(json.dumps(rec), flush=True)
    comm.destroy()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
