#!/usr/bin/env python3
"""BASELINE config 4: MAG240M-shaped R-GCN, full-graph training step.

One process per GPU (torchrun for N > 1). Synthetic MAG240M-shaped heterogeneous graph
(121.75M papers, 122.38M authors, 25.7K institutions; 1.30B citations symmetrised, 386M
writes, 44.6M affiliations, each in both directions; 768 features, 153 classes; random
features and weights), generated per rank on the device (``dgraph_amd.data.mag``).
A step = forward of every (layer, node type) that reaches the paper loss, masked
cross-entropy over the train papers, backward, gradient all-reduce, Adam.

Layer 0 reads its halo feature rows ONCE: with ``--backend rocshmem`` the features live
on the HIP-IPC symmetric heap and each rank fetches its halo rows with the one-sided
remote-get kernel (the reference's NVSHMEM ``dist_get``); with ``nccl`` by one RCCL
all-to-all-v. Later layers exchange hidden-activation halos per step (RCCL, overlapped).

The whole MAG240M-shaped graph needs ~8 GPUs; on one GPU use ``--scale 0.125`` (one
eighth of every count: the per-GPU share of the 8-GPU job) or ``--rehearse-world 8``
(rank ``--rehearse-rank`` of the real 8-way partition, halo included, loopback exchange).

    edges_per_s = (messages aggregated per step, summed over the computed relations) / step_s
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# (no max_split_size here, unlike bench.py: the relation tensors come in many different
#  large sizes, and unsplittable cached blocks then miss on almost every request —
#  hipMalloc/hipFree churn took a W=8 rank's step from 476 ms to 3.1 s)

import torch
import torch.distributed as dist
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--shape", default="mag240m")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--dropout", type=float, default=0.5)
    ap.add_argument("--global-frac", type=float, default=0.05)
    ap.add_argument("--window", type=int, default=1 << 14)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "rocshmem", "nvshmem"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--rehearse-world", type=int, default=0)
    ap.add_argument("--rehearse-rank", type=int, default=0)
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32",
                    help="compute/storage dtype (fp32 = the reference's precision: "
                         "experiments/OGB-LSC/RGAT.py has no casts; bf16 = autocast with fp32 "
                         "master weights, a secondary)")
    ap.add_argument("--path", choices=("auto", "lean", "aggregate-first"), default="auto",
                    help="R-GCN execution path (auto: lean at fp32, aggregate-first under bf16)")
    ap.add_argument("--link-gbps", type=float, default=0.0,
                    help="rehearsal link model: every loopback exchange takes latency + "
                         "largest per-peer message / GBPS (comm/alltoallv.py); the step-time "
                         "difference to --link-gbps 0 is the exchange time the schedule "
                         "exposes")
    ap.add_argument("--model", choices=("rgcn", "rgat"), default="rgcn",
                    help="rgat: the reference's OGB-LSC model (experiments/OGB-LSC/RGAT.py) on "
                         "its lean fp32 path (fused relation attention, ops/gat.py)")
    ap.add_argument("--heads", type=int, default=4,
                    help="RGAT attention heads (the reference config's 4)")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args(argv)


def log(rank, *a):
    if rank == 0:
        print("[bench_rgcn]", *a, file=sys.stderr, flush=True)


def main(argv=None):
    args = parse(argv)
    if args.link_gbps > 0:
        import dgraph_amd.comm.alltoallv as _A

        _A.LOOPBACK_LINK_GBPS = args.link_gbps
    from dgraph_amd import Communicator
    from dgraph_amd.data.mag import (EDGE_TYPES, HETERO_SHAPES, build_hetero_partition,
                                     hetero_node_data)
    from dgraph_amd.models.rgcn import CommAwareRGCN, HeteroGraph, layer_plan
    from dgraph_amd.parallel.grad_sync import GradSync

    comm = Communicator.init_process_group(args.backend)
    rank, world = comm.get_rank(), comm.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")
    shape = HETERO_SHAPES[args.shape]
    if args.scale != 1.0:
        shape = shape.scaled(args.scale)
    rehearse = args.rehearse_world > 1 and world == 1
    p_rank, p_world = (args.rehearse_rank, args.rehearse_world) if rehearse else (rank, world)
    _, rels_used = layer_plan(EDGE_TYPES, args.layers, 0)
    needed = sorted({r for rs in rels_used for r in rs})
    t0 = time.time()
    part = build_hetero_partition(shape, p_rank, p_world, dev, seed=args.seed,
                                  global_frac=args.global_frac, window=args.window,
                                  group=comm.group, rehearse=rehearse, relations=needed)
    graph = HeteroGraph.from_partition(part, EDGE_TYPES, group=comm.group, rank=p_rank)
    dtype = torch.bfloat16 if (dev.type == "cuda" and args.dtype == "bf16") else torch.float32
    heap = None
    alloc = None
    if args.backend != "nccl" and dev.type == "cuda" and p_world > 1 and not rehearse:
        # features on the symmetric heap (same offset on every rank: sized to the max rows)
        from dgraph_amd.comm.symheap import SymmetricHeap

        offs = part["offsets"]
        need_b = 0
        for t in range(3):
            n_max = max(offs[t][r + 1] - offs[t][r] for r in range(p_world))
            need_b += (n_max * shape.num_features * torch.empty((), dtype=dtype).element_size()
                       + 511) // 256 * 256
        heap = SymmetricHeap(need_b + (1 << 20), comm.group)

        def alloc(t, shp, dt, _o=offs):
            n_max = max(_o[t][r + 1] - _o[t][r] for r in range(p_world))
            return heap.alloc_tensor((n_max, shp[1]), dt)[: shp[0]]

        for sg in graph.sources.values():
            sg.heap = heap
    feats, y, train = hetero_node_data(shape, p_rank, part["offsets"], dev, seed=args.seed,
                                       dtype=dtype, alloc=alloc)
    if args.model != "rgat":  # (RGAT's patterns carry their own transposes, ops/gat.py)
        for sg in graph.sources.values():
            sg.prepare_backward()
    train_idx = torch.nonzero(train, as_tuple=True)[0]
    y_train = y[train_idx]
    del y, train
    # messages aggregated per step, per layer over the computed relations
    nnz = {}
    for sg in graph.sources.values():
        for r, (lo, hi) in sg.ranges.items():
            n = int(sg.interior.rowptr[hi] - sg.interior.rowptr[lo])
            if sg.halo is not None:
                n += int(sg.halo.rowptr[hi] - sg.halo.rowptr[lo])
            nnz[r] = n
    msgs = sum(nnz[r] for rs in rels_used for r in rs)
    e_local = torch.tensor([msgs, train_idx.numel(),
                            sum(sg.H for sg in graph.sources.values())],
                           dtype=torch.long, device=dev)
    if world > 1:
        dist.all_reduce(e_local)
    E_step, n_train, halo_total = (int(v) for v in e_local.tolist())
    log(rank, f"graph built in {time.time() - t0:.1f}s: nodes={shape.num_nodes} "
              f"messages/step={E_step} halo_rows={halo_total} train={n_train}")

    torch.manual_seed(args.seed)
    if args.model == "rgat":
        from dgraph_amd.models.rgat import CommAwareRGAT

        if dtype != torch.float32:
            raise SystemExit("[bench_rgcn] --model rgat runs the lean fp32 path only")
        model = CommAwareRGAT(shape.num_features, shape.num_classes, args.hidden,
                              len(EDGE_TYPES), args.layers, args.heads, comm=comm,
                              dropout=args.dropout, bn_group=comm.group).to(dev)
    else:
        model = CommAwareRGCN(shape.num_features, args.hidden, shape.num_classes,
                              len(EDGE_TYPES), args.layers, dropout=args.dropout, comm=comm,
                              bn_group=comm.group).to(dev)
        if args.path != "auto":
            model.lean = args.path == "lean"
    opt = torch.optim.Adam(model.parameters(), lr=args.lr, fused=dev.type == "cuda")
    sync = GradSync(model.parameters(), group=comm.group) if world > 1 else None
    inv_n = 1.0 / max(n_train, 1)
    use_amp = dev.type == "cuda" and dtype == torch.bfloat16

    lean = True if args.model == "rgat" else (
        model.lean if model.lean is not None else (dtype == torch.float32))

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=use_amp):
            logits = model(feats, graph)
        loss = F.cross_entropy(logits[train_idx].float(), y_train, reduction="sum") * inv_n
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
    def alloc_stats():
        if dev.type != "cuda":
            return {}
        st = torch.cuda.memory_stats(dev)
        return {k: int(st.get(k, 0)) for k in ("num_device_alloc", "num_device_free",
                                                "num_alloc_retries")}

    a0 = alloc_stats()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        l = step()
    barrier_sync()
    a1 = alloc_stats()
    alloc_timed = {k: a1[k] - a0[k] for k in a0}
    ms = torch.tensor([(time.perf_counter() - t1) * 1e3 / max(args.steps, 1)],
                      dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    ms_step = float(ms.item())
    lt = l.detach().reshape(1).double()
    if world > 1:
        dist.all_reduce(lt)
    peak = torch.cuda.max_memory_allocated() / 1e9 if dev.type == "cuda" else 0.0
    rec = {
        "metric": "edges_per_s", "value": E_step / (ms_step / 1e3), "unit": "edges/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
        "epoch_ms": ms_step, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
        "data": (f"synthetic {shape.name}-shaped hetero graph (nodes={list(shape.num_nodes)}, "
                 f"global_frac={args.global_frac}, window={args.window}), random features/"
                 f"labels, random-init weights"),
        "config": {"model": (f"RGAT {args.layers}-layer hidden {args.hidden} heads "
                             f"{args.heads}" if args.model == "rgat" else
                             f"R-GCN {args.layers}-layer hidden {args.hidden}"),
                   "backend": args.backend, "messages_per_step": E_step,
                   "halo_rows_total": halo_total, "train_papers": n_train,
                   "parallelism": f"graph-partition{p_world}" + (" (rehearsal)" if rehearse
                                                                  else "")},
        "final_loss": float(lt.item()), "peak_mem_gb_rank0": round(peak, 2),
        "path": "lean" if lean else "aggregate-first",
        "layer0_halo": ("kept" if (not lean or
                                   CommAwareRGCN._keep_static_halo(model, feats, graph))
                        else "exchanged per step"),
        "allocator_in_timed_steps": alloc_timed,
    }
    if rehearse:
        rec = {"rehearsal": True, "model": rec["config"]["model"], "rank": p_rank,
               "world": p_world,
               "ms_per_step_compute_loopback": ms_step, "messages_local": E_step,
               "halo_rows": halo_total, "peak_mem_gb": round(peak, 2),
               "final_loss_local": float(lt.item()), "path": rec["path"],
               "layer0_halo": rec["layer0_halo"], "link_gbps": args.link_gbps,
               "allocator_in_timed_steps": alloc_timed,
               "backend": args.backend,
               "dtype": "bf16" if dtype == torch.bfloat16 else "fp32"}
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if heap is not None:
        heap.close()
    comm.destroy()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
