#!/usr/bin/env python3
"""Headline benchmark: full-graph GraphSAGE training on an ogbn-papers100M-shaped graph.

BASELINE.json metric: "edges/sec + epoch time, ogbn-papers100M 3-layer GraphSAGE at
1/2/4/8 MI355X". One process per GPU (torchrun), vertex-partitioned graph (contiguous
partition of a synthetic graph with the papers100M shape: 111,059,956 nodes,
1,615,685,872 directed edges symmetrised to ~3.23B messages per layer, 128 features,
172 classes), RCCL all-to-all-v halo exchange overlapped with interior aggregation.

A step is the reference's full-graph epoch (experiments/OGB/main.py:129-184):
  forward of ALL 3 SAGE-mean layers over ALL vertices (hidden 256, fp32 — the reference's
  precision — on the memory-lean row-chunked executor models/sage_fused.py) -> masked
  cross-entropy on the train split, and validation/test accuracy from the SAME forward ->
  backward -> gradient all-reduce -> Adam step.
The output layer's backward uses only the train rows' nonzero gradient (A[train, :]^T),
and the layer below it aggregates transposed only from the rows where its incoming
gradient can be nonzero (the train rows and their neighbours, DistGraph.grad_support):
exact (the dense backward multiplies zeros), counted as what it aggregates.

    value = edges_per_s = num_layers * E_msg / step_s      (BASELINE.md §2 definition)
    edges_aggregated_per_step = nonzeros actually aggregated, forward + backward

Secondary measurements in the same JSON line (unless --no-extra):
  * "structureless": the same step on a --global-frac 1.0 graph (uniformly random
    endpoints: no locality for any cache to exploit);
  * "bf16_stack": the headline graph at bf16 storage/compute on the layer-stack path
    (below the reference's precision; labelled, never the headline);
  * "train_rows_only" (layer-stack executor only): the step with the output layer
    aggregated only at the train rows (not a full-graph forward; never the headline).
  * "regions": per-region device ms of one extra step (max/min over ranks), exposed
    exchange vs compute, bytes per peer (the reference's TimingReport regions).
The whole graph is fixed as N grows (strong scaling). Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

# large, long-lived activations + transient SpMM buffers: avoid allocator fragmentation
# (expandable segments are unsupported on ROCm; forbid splitting huge cached blocks so a
#  freed 57 GB activation block is never carved up by a 38 GB request)
os.environ.setdefault("PYTORCH_ALLOC_CONF", "max_split_size_mb:512")
# hardware queues per process: left as the box exports them (HIP's default, 4) — the halo
# exchange rides a high-priority stream, which gets a queue of its own at any queue budget
# (comm/alltoallv.py _side_stream); the value in effect is recorded in the JSON line
_HWQ_FOUND = os.environ.get("GPU_MAX_HW_QUEUES")

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
    ap.add_argument("--dtype", choices=("bf16", "fp32"), default="fp32",
                    help="compute/storage dtype of features and activations; fp32 (default) "
                         "is the reference's precision (weights are fp32 masters either way)")
    ap.add_argument("--executor", choices=("auto", "fused", "stack"), default="auto",
                    help="fused: the memory-lean fp32 row-chunked executor "
                         "(models/sage_fused.py; fits papers100M fp32 on one GPU); stack: the "
                         "layer-stack autograd node (models/sage.py SAGEStackFn); auto = fused "
                         "for fp32 shapes it supports")
    ap.add_argument("--no-bf16-extra", action="store_true",
                    help="skip the secondary bf16 (layer-stack) measurement of the headline graph")
    ap.add_argument("--plan-reserve-gb", type=float, default=None,
                    help="GB the fused executor's memory plan leaves free (default: 24 for the "
                         "structureless extra at W > 1, else 0)")
    ap.add_argument("--global-frac", type=float, default=0.05,
                    help="fraction of uniformly random (non-local) edges of the headline "
                         "graph; the rest join ids within +-window")
    ap.add_argument("--window", type=int, default=1 << 14)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--restrict-last", action="store_true",
                    help="headline = train-rows-only step (output layer aggregated at the "
                         "train rows only); NOT a full-graph step, for A/B only")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the structureless-graph and train-rows-only measurements")
    ap.add_argument("--extra-steps", type=int, default=3)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--rehearse-world", type=int, default=0,
                    help="single process: run rank --rehearse-rank of a W-way partition with "
                         "a loopback halo exchange (per-rank compute + memory; no peers)")
    ap.add_argument("--rehearse-rank", type=int, default=0)
    ap.add_argument("--link-gbps", type=float,
                    default=float(os.environ.get("DGRAPH_LOOPBACK_LINK_GBPS", "0")),
                    help="rehearsal: hold each loopback exchange for latency + largest "
                         "per-peer message / GBPS (one xGMI link per peer pair) on a side "
                         "stream, so the exposed-exchange regions measure the overlap "
                         "schedule against link-length transfers (0 = instant loopback)")
    ap.add_argument("--link-cus", type=int, default=-1,
                    help="rehearsal link model: CUs the modelled collective holds during a "
                         "transfer (default DGRAPH_LOOPBACK_CUS = 16)")
    ap.add_argument("--no-interior-first", dest="interior_first", action="store_false",
                    help="W>1 fused executor: keep the original row order (no interior-first "
                         "renumbering, parallel/reorder.py)")
    ap.add_argument("--profile-ops", default="",
                    help="after the timed steps, profile one extra step (every rank runs it) "
                         "with torch.profiler; rank 0 writes the per-op device-time table")
    ap.add_argument("--halo-recompute", choices=("auto", "on", "off"), default="auto",
                    help="W>1: compute the first hidden layer for the halo vertices too, so "
                         "layer 2 exchanges nothing forward or backward "
                         "(parallel/halo_recompute.py); auto = on when every rank's halo "
                         "is smaller than its partition")
    ap.add_argument("--cuda-graph", action="store_true",
                    help="capture the whole step (forward, backward, sync, Adam) into a HIP "
                         "graph after the first eager warmup step and replay it "
                         "(dgraph_amd.utils.graphed; for launch-bound small shapes)")
    ap.add_argument("--no-shmem-probe", action="store_true",
                    default=os.environ.get("DGRAPH_BENCH_SHMEM_PROBE", "1") == "0",
                    help="W > 1: skip the one-sided (symmetric-heap) transport probe that runs "
                         "as a separate child job after the headline")
    ap.add_argument("--shmem-probe-timeout", type=float,
                    default=float(os.environ.get("DGRAPH_BENCH_SHMEM_PROBE_TIMEOUT_S", "150")))
    ap.add_argument("--metrics-jsonl", default=os.environ.get("DGRAPH_METRICS_JSONL", ""),
                    help="append one metrics record per measured phase (rank 0)")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def _profile_one_step(step, path, rank):
    """Per-aten-op device time of one (untimed) step, grouped by input shape. Every rank
    runs the step (its collectives must match); rank 0 writes the table."""
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    if rank == 0:
        ka = prof.key_averages(group_by_input_shape=True)
        with open(path, "w") as f:
            f.write(ka.table(sort_by="self_cuda_time_total", row_limit=60,
                             max_name_column_width=60, max_shapes_column_width=90))


class Job:
    """One graph + data + model + optimizer on this rank (built collectively)."""

    def __init__(self, args, comm, dev, global_frac: float, dtype):
        from dgraph_amd.data.synthetic import (SHAPES, SPLIT_TEST, SPLIT_TRAIN, SPLIT_VALID,
                                               build_partition, node_data)
        from dgraph_amd.models.sage import GraphSAGE
        from dgraph_amd.parallel.dist_graph import DistGraph
        from dgraph_amd.parallel.grad_sync import GradSync

        self.args, self.dev = args, dev
        self.rank, self.world = comm.get_rank(), comm.get_world_size()
        shape = SHAPES[args.shape]
        if args.scale != 1.0:
            shape = shape.scaled(args.scale)
        self.shape = shape
        self.global_frac = global_frac
        t0 = time.time()
        self.rehearse = args.rehearse_world > 1 and self.world == 1
        p_rank, p_world = ((args.rehearse_rank, args.rehearse_world) if self.rehearse
                           else (self.rank, self.world))
        self.p_rank, self.p_world = p_rank, p_world
        part = build_partition(shape, p_rank, p_world, dev, seed=args.seed,
                               global_frac=global_frac, window=args.window,
                               rehearse=self.rehearse)
        ex = getattr(args, "executor", "auto")
        from dgraph_amd.models.sage_fused import HIDDEN_WIDTHS

        self.use_fused = ex == "fused" or (ex == "auto" and dtype == torch.float32 and
                                           args.layers in (2, 3) and
                                           args.hidden in HIDDEN_WIDTHS)
        csr = part["csr"]
        if p_world == 1:
            csr.num_cols = part["L"]
        self.L, self.H = part["L"], part["H"]
        # W > 1, fused executor: number this rank's rows interior-first (rows with no halo
        # neighbour and sent to nobody first), so each layer's interior rows run while its
        # halo exchange is in flight (parallel/reorder.py); per-vertex data follows perm
        self.perm, locality = None, None
        if p_world > 1 and self.use_fused and getattr(args, "interior_first", True):
            from dgraph_amd.parallel.reorder import interior_first

            csr, part["send_local_idx"], self.perm, self.L_int, locality = interior_first(
                csr, part["L"], part["send_local_idx"])
            part["csr"] = csr
        self.graph = DistGraph(csr, part["L"], part["H"], part["send_local_idx"],
                               part["send_splits"],
                               # the synthetic graph is symmetrised, so the interior
                               # (local x local) block is symmetric at every W: its
                               # transpose is never materialised
                               part["recv_splits"], comm.group, symmetric=True,
                               overlap=not args.no_overlap)
        if locality is not None:
            self.graph.locality_hint = locality
        halo_gids = part["halo_gids"]
        del part, csr
        if not self.use_fused:
            self.graph.prepare_backward()
        self.recompute = False
        mode = getattr(args, "halo_recompute", "off")
        if p_world > 1 and mode != "off" and args.layers >= 3 and not self.use_fused:
            want = torch.tensor([1 if (mode == "on" or self.H < self.L) else 0],
                                dtype=torch.long, device=dev)
            if self.world > 1:
                dist.all_reduce(want, op=dist.ReduceOp.MIN)  # one decision for all ranks
            if int(want) == 1:
                from dgraph_amd.data.synthetic import build_rows_csr
                from dgraph_amd.parallel.halo_recompute import HaloRecompute

                rows_csr = build_rows_csr(shape, halo_gids, dev, seed=args.seed,
                                          global_frac=global_frac, window=args.window)
                self.graph.recompute = HaloRecompute(
                    self.graph, rows_csr, halo_gids, _offsets(shape.num_nodes, p_world),
                    p_rank, comm.group, rehearse=self.rehearse)
                del rows_csr
                self.recompute = True
        del halo_gids
        self.x, y, split = node_data(shape, p_rank,
                                     _offsets(shape.num_nodes, p_world), dev, seed=args.seed,
                                     dtype=dtype, return_split=True)
        if self.perm is not None:
            self.x, y, split = self.x[self.perm], y[self.perm], split[self.perm]
            self.perm = None
        self.train_idx = torch.nonzero(split == SPLIT_TRAIN, as_tuple=True)[0]
        # the gradient support of the layer below the output layer
        # (DistGraph.prepare_grad_support), built now while device memory is free
        # (collective: every rank builds it at this point); DGRAPH_BENCH_GRAD_SUPPORT=off
        # for the A/B
        gs = os.environ.get("DGRAPH_BENCH_GRAD_SUPPORT", "on")
        if args.layers >= 2 and gs != "off" and not self.use_fused:
            self.graph.prepare_grad_support(self.train_idx)
        self.y_train = y[self.train_idx]
        ev = split == SPLIT_VALID
        ev |= split == SPLIT_TEST
        self.eval_idx = torch.nonzero(ev, as_tuple=True)[0]
        self.y_eval = y[self.eval_idx]
        self.eval_is_val = (split[self.eval_idx] == SPLIT_VALID)
        del y, split, ev
        cnt = torch.tensor([self.graph.nnz, self.train_idx.numel(), self.H,
                            int(self.eval_is_val.sum()),
                            self.eval_idx.numel()], dtype=torch.long, device=dev)
        if self.world > 1:
            dist.all_reduce(cnt)
        self.E_msg, self.n_train, self.halo_total, self.n_val, n_eval = (
            int(v) for v in cnt.tolist())
        self.n_test = n_eval - self.n_val
        self.build_s = time.time() - t0
        torch.manual_seed(args.seed)
        self.model = GraphSAGE(shape.num_features, args.hidden, shape.num_classes,
                               args.layers).to(dev)
        self.opt = torch.optim.Adam(self.model.parameters(), lr=args.lr,
                                    fused=dev.type == "cuda")
        self.fused = None
        if self.use_fused:
            from dgraph_amd.models.sage_fused import FusedSAGE, supported

            if dev.type == "cuda":
                gc.collect()  # the build's cached blocks back before the workspace is sized
                torch.cuda.empty_cache()

            if not supported(self.model, self.x):
                raise SystemExit("[bench] --executor fused does not support this shape/dtype")
            # a secondary graph (the structureless extra) at W > 1 plans with 24 GB of
            # headroom: its halo sizes differ from rank to rank, and an OOM on one rank
            # mid-step would take the whole job (and its headline line) down
            reserve = (24 << 30) if (global_frac != args.global_frac and self.world > 1) else 0
            if getattr(args, "plan_reserve_gb", None) is not None:
                reserve = int(args.plan_reserve_gb * (1 << 30))
            self.fused = FusedSAGE(self.model, self.graph, self.x, self.train_idx, self.y_train,
                                   self.eval_idx, self.y_eval, self.eval_is_val, self.n_train,
                                   release_graph=True, reserve_bytes=reserve,
                                   config=getattr(args, "exec_cfg", None))
        self.steppers = {}
        if getattr(args, "cuda_graph", False) and dev.type == "cuda":
            from dgraph_amd.utils.graphed import GraphedStep, make_capturable

            make_capturable(self.opt)
            self.steppers = {r: GraphedStep(lambda r=r: self.step(r), warmup=1)
                             for r in (False, True)}
        self.sync = GradSync(self.model.parameters(), group=None) if self.world > 1 else None
        if dev.type == "cuda":
            # return the graph build's cached temporaries (blocks > 512 MB are never split:
            # left cached they pin tens of GB the training workspace cannot reuse, and the
            # libraries' own device allocations then find no free memory)
            gc.collect()
            torch.cuda.empty_cache()
        self.inv_n = 1.0 / max(self.n_train, 1)
        self.correct = torch.zeros(2, dtype=torch.long, device=dev)  # val, test
        # resident after setup (graph, data, activations, workspace): the timed steps'
        # peak minus this is the step's transient memory
        self.mem_setup_gb = torch.cuda.memory_allocated(dev) / 1e9 if dev.type == "cuda" \
            else 0.0

    def step(self, restrict_last: bool = False):
        import torch.nn.functional as Fn

        g = self.graph
        if self.fused is not None:
            # fp32 row-chunked executor: loss, p.grad and val/test hits of one full-graph step
            loss = self.fused.step()
            self.correct.copy_(self.fused.correct)
            if self.sync is not None:
                self.sync.all_reduce()
            self.opt.step()
            return loss
        if restrict_last:
            logits = self.model(self.x, g, out_rows=self.train_idx, restrict_last=True)
        else:
            logits, ev = self.model(self.x, g, out_rows=self.train_idx,
                                    eval_rows=self.eval_idx)
            # validation/test accuracy from the same forward (device counters, no sync)
            hit = ev.argmax(1) == self.y_eval
            self.correct[0] = (hit & self.eval_is_val).sum()
            self.correct[1] = (hit & ~self.eval_is_val).sum()
        loss = Fn.cross_entropy(logits.float(), self.y_train, reduction="sum") * self.inv_n
        loss.backward()
        if self.sync is not None:
            self.sync.all_reduce()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        return loss

    def stepper(self, restrict_last: bool):
        """The step as a callable: eager, or captured once and replayed (--cuda-graph)."""
        return self.steppers.get(restrict_last) or (lambda: self.step(restrict_last))

    def halo_stats(self):
        from dgraph_amd.utils.diagnostics import halo_stats

        if self.world == 1 and not self.rehearse:
            return {}
        fb = self.args.hidden * self.x.element_size()
        st = halo_stats(self.graph, fb)
        keep = ("max_pairwise_bytes", "max_rank_send_bytes", "xgmi_bound_ms")
        out = {k: st[k] for k in keep if k in st}
        # full-width exchanges of one training step (the output layer's restricted
        # backward exchange, ~1 % of rows, not counted): hidden-layer halos forward and
        # backward, the projected output layer forward; only the latter with recompute
        from dgraph_amd.models.sage import _pad_width

        c_out = _pad_width(self.shape.num_classes)
        if self.fused is not None:
            # hidden activations forward (layers - 1) + layer 0's reverse exchange
            widths = [self.args.hidden] * (self.args.layers - 1) + \
                ([self.args.hidden] if self.args.layers == 3 else [])
        elif self.recompute:
            widths = [c_out]
        else:
            widths = [self.args.hidden] * (self.args.layers - 2) + [c_out] + \
                [self.args.hidden] * (self.args.layers - 2)
        out["exchange_widths_per_step"] = widths
        if "max_pairwise_bytes" in out:
            rows = out["max_pairwise_bytes"] / fb
            out["max_pairwise_bytes_per_step"] = rows * sum(widths) * self.x.element_size()
        return out

    def free(self):
        for k in ("fused", "graph", "x", "model", "opt", "sync", "train_idx", "y_train",
                  "eval_idx", "y_eval", "eval_is_val"):
            setattr(self, k, None)


def _link_cus():
    from dgraph_amd.comm import alltoallv as _a2a

    return _a2a.LOOPBACK_CUS


def _offsets(n, w):
    from dgraph_amd.data.synthetic import contiguous_offsets

    return contiguous_offsets(n, w)


def barrier_sync(world, dev):
    if world > 1:
        dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()


def _alloc_counters(dev) -> dict:
    """Caching-allocator counters: hipMalloc/hipFree calls and allocation retries."""
    if dev.type != "cuda":
        return {"num_device_alloc": 0, "num_device_free": 0, "num_alloc_retries": 0}
    s = torch.cuda.memory_stats(dev)
    return {k: int(s.get(k, 0)) for k in ("num_device_alloc", "num_device_free",
                                          "num_alloc_retries")}


def timed(job: Job, steps: int, warmup: int, restrict_last: bool, verbose: bool = False):
    """W untimed warmup steps, then K steps bracketed by barrier + synchronize; returns
    (ms_per_step as the MAX over ranks, mean loss of the last step summed over ranks,
     edges aggregated per step summed over ranks)."""
    world, dev = job.world, job.dev
    stepf = job.stepper(restrict_last)
    e_eager = None  # edges of one step, counted on the host while the step's Python runs
    for i in range(warmup):
        ea = job.graph.edges_aggregated
        l = stepf()
        if e_eager is None:
            e_eager = job.graph.edges_aggregated - ea
        if verbose:
            log(job.rank, f"warmup {i} loss {float(l.detach()):.4f}")
    barrier_sync(world, dev)
    a0 = _alloc_counters(dev)
    e0 = job.graph.edges_aggregated
    t_start = time.perf_counter()
    l = None
    for _ in range(steps):
        l = stepf()
    barrier_sync(world, dev)
    elapsed = time.perf_counter() - t_start
    a1 = _alloc_counters(dev)
    job.alloc_timed = {k: a1[k] - a0[k] for k in a0 if k.startswith("num_")}
    if dev.type == "cuda":
        job.alloc_timed["reserved_minus_allocated_gb"] = round(
            (torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)) / 1e9, 3)
    e1 = job.graph.edges_aggregated
    if job.steppers and e_eager is not None:
        # graph replays run no Python, so the host counter did not move: every replay
        # aggregates what the captured (eager-equivalent) step did
        e1 = e0 + e_eager * steps
    red = torch.tensor([elapsed * 1000.0 / max(steps, 1)], dtype=torch.float64, device=dev)
    tot = torch.tensor([float(l.detach()) if l is not None else 0.0,
                        (e1 - e0) / max(steps, 1)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(red, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot)  # each rank holds its share of the global mean loss
    return float(red.item()), float(tot[0].item()), float(tot[1].item())


def link_probe(job: "Job", width: int = 64, iters: int = 5) -> dict:
    """Achieved xGMI bandwidth of this job's own halo exchange (W > 1, every rank, after
    the timed steps): the plan's all-to-all-v of ``width`` fp32 columns, ``iters`` times
    back to back between barriers, timed with stream events; per rank the largest
    per-peer message over the exchange time is the per-link rate its slowest link
    delivered. Reduced to max / min over ranks. (The rehearsal's link model assumes
    153 GB/s per link; this is the measured number.)"""
    g = job.graph
    a2a = getattr(g, "a2a", None)
    if job.world <= 1 or a2a is None or job.dev.type != "cuda":
        return {}

    def view(t, n):  # a contiguous [n, width] block of a resident buffer, if large enough
        return t.view(-1)[:n * width].view(n, width) if t is not None and \
            t.is_contiguous() and t.numel() >= n * width else None

    ex = job.fused
    send = view(getattr(ex, "send_buf", None), a2a.total_send)
    recv = view((getattr(ex, "halo_buf", None) or [None])[0], a2a.total_recv)
    ok = 1
    try:  # (resident exchange buffers of the executor when it has them, else fresh)
        if send is None:
            send = torch.empty(a2a.total_send, width, device=job.dev)
        if recv is None:
            recv = torch.empty(a2a.total_recv, width, device=job.dev)
        gen = torch.Generator(device=job.dev)
        gen.manual_seed(1234 + job.rank)
        send.uniform_(generator=gen)  # distinct rows: the executor A/B compares them bitwise
    except torch.OutOfMemoryError:
        ok = 0
    okt = torch.tensor([ok], device=job.dev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)  # every rank probes, or none does
    if int(okt) == 0:
        return {"skipped": "no device memory for the probe buffers"}
    for _ in range(2):
        a2a(send, out=recv)
    torch.cuda.synchronize()
    dist.barrier()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        a2a(send, out=recv)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    peer = max(max(a2a.send_splits, default=0), max(a2a.recv_splits, default=0)) * width * 4
    tot = (a2a.total_send + a2a.total_recv) * width * 4
    v = torch.tensor([ms, peer / (ms * 1e6), tot / (ms * 1e6)], dtype=torch.float64,
                     device=job.dev)
    vmax, vmin = v.clone(), v.clone()
    dist.all_reduce(vmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(vmin, op=dist.ReduceOp.MIN)
    impl = os.environ.get("DGRAPH_A2A_IMPL", "torch")
    nat = native_probe(job, a2a, send, recv, iters) \
        if impl == "torch" and dist.get_backend(a2a.group) == "nccl" else {}
    del send, recv
    return {"columns": width, "exchange_ms_max": round(float(vmax[0]), 3),
            "largest_peer_message_GBps_min_over_ranks": round(float(vmin[1]), 1),
            "largest_peer_message_GBps_max_over_ranks": round(float(vmax[1]), 1),
            "rank_send_plus_recv_GBps_min_over_ranks": round(float(vmin[2]), 1),
            "transport": impl, **({"native_executor": nat} if nat else {})}


def native_probe(job: "Job", a2a, send: torch.Tensor, ref: torch.Tensor, iters: int) -> dict:
    """The same exchange through the native grouped send/recv executor (comm/rccl_exec.py:
    its own RCCL communicator, host-cached splits, zero-size peers skipped) right after the
    torch-PG one: bitwise equality of the received rows with ``ref`` (what the torch path
    received) on every rank, and its exchange time. The executor's communicator is
    destroyed afterwards (its buffers do not stay resident for the secondaries)."""
    from dgraph_amd.comm.rccl_exec import RCCLExecutor

    ok = 1
    try:
        out = torch.empty_like(ref)
    except torch.OutOfMemoryError:
        ok = 0
    okt = torch.tensor([ok], device=job.dev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    if int(okt) == 0:
        return {"skipped": "no device memory for a second receive buffer"}
    ex = RCCLExecutor.for_group(a2a.group)
    try:
        for _ in range(2):
            ex.alltoallv([send], [out], a2a.send_splits, a2a.recv_splits)
        torch.cuda.synchronize()
        eq = torch.tensor([1 if torch.equal(out, ref) else 0], device=job.dev)
        dist.barrier()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            ex.alltoallv([send], [out], a2a.send_splits, a2a.recv_splits)
        e.record()
        torch.cuda.synchronize()
        ms = torch.tensor([s.elapsed_time(e) / iters], dtype=torch.float64, device=job.dev)
        dist.all_reduce(eq, op=dist.ReduceOp.MIN)
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    finally:
        RCCLExecutor.close_all()
    del out
    return {"bitwise_equal_to_torch": bool(int(eq) == 1),
            "exchange_ms_max": round(float(ms), 3)}


def region_breakdown(job: "Job") -> dict:
    """One extra (untimed) step with stream events at the executor's region boundaries:
    per-region device ms on every rank (no barrier or host sync inside the step), reduced
    to max / min over ranks, plus the halo bytes each rank sent per peer during that step
    and the achieved bytes per second over its exposed exchange time."""
    ex = job.fused
    if ex is None:
        return {}
    from dgraph_amd.comm.alltoallv import CommStats

    CommStats.reset()
    ex.record = True
    job.step()
    ex.record = False
    reg = ex.region_ms()
    sent = dict(CommStats.peer_bytes_sent)
    names = sorted(reg)
    exch = sum(v for k, v in reg.items() if k.startswith("exchange"))
    comp = sum(v for k, v in reg.items() if not k.startswith("exchange"))
    vals = [reg[k] for k in names] + [comp, exch]
    world = job.world
    if world > 1:
        names_all = [None] * world
        dist.all_gather_object(names_all, names)
        if any(n != names for n in names_all):
            return {"error": "ranks recorded different regions"}
        t = torch.tensor(vals, dtype=torch.float64, device=job.dev)
        tmax, tmin = t.clone(), t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(tmin, op=dist.ReduceOp.MIN)
        sent_all = [None] * world
        dist.all_gather_object(sent_all, sent)
        tmax, tmin = tmax.tolist(), tmin.tolist()
    else:
        tmax = tmin = vals
        sent_all = [sent]
    out = {
        "ms_max_over_ranks": {k: round(v, 3) for k, v in zip(names, tmax)},
        "ms_min_over_ranks": {k: round(v, 3) for k, v in zip(names, tmin)},
        "compute_ms_max": round(tmax[-2], 3), "compute_ms_min": round(tmin[-2], 3),
        "exposed_exchange_ms_max": round(tmax[-1], 3),
        "exposed_exchange_ms_min": round(tmin[-1], 3),
    }
    if world > 1:
        per_peer = [max(d.values()) if d else 0 for d in sent_all]
        out["max_bytes_per_peer_per_step"] = max(per_peer)
        out["bytes_sent_per_rank"] = [int(sum(d.values())) for d in sent_all]
        if tmax[-1] > 0:
            out["achieved_peer_GBps_over_exposed_exchange"] = round(
                max(per_peer) / (tmax[-1] / 1e3) / 1e9, 2)
    return out


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def shmem_probe_child(args, rank: int, world: int, splits, dev) -> dict:
    """The one-sided transport probe (dgraph_amd/comm/shmem_probe.py) over the headline's
    own halo plan, as a SEPARATE JOB: every rank starts one child process (a fresh
    interpreter on the same GPU, its own process group on a new port) and waits for it; the
    ranks themselves are never replaced and run nothing on the GPU meanwhile. A fault, a
    hang (killed at ``--shmem-probe-timeout``) or an error in any child is recorded as
    ``{"failed": ...}``; the headline line is printed either way. The children's outcome is
    gathered over a CPU (gloo) group, which a GPU fault in a child cannot disturb. Returns
    the merged record on rank 0 ({} elsewhere)."""
    import subprocess
    import tempfile

    cpu = dist.new_group(backend="gloo")  # collective: every rank
    port = [_free_port() if rank == 0 else 0]
    dist.broadcast_object_list(port, src=0, group=cpu)
    fd, path = tempfile.mkstemp(prefix=f"dgraph_shmem_plan_r{rank}_", suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump({"send_splits": splits[0], "recv_splits": splits[1]}, f)
    env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_RANK=os.environ.get("LOCAL_RANK", str(rank)), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port[0]),
               DGRAPH_PG_TIMEOUT_S=str(int(max(30, args.shmem_probe_timeout * 0.5))))
    # torchrun's agent store is not the child's rendezvous: rank 0's child hosts its own
    for k in ("TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_RUN_ID", "GROUP_RANK",
              "ROLE_RANK", "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS"):
        env.pop(k, None)
    if dev.type == "cuda":
        gc.collect()
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()  # the headline's cached blocks back for the child
    cmd = [sys.executable, "-u", "-m", "dgraph_amd.comm.shmem_probe", "--plan", path,
           "--width", "64", "--iters", "5"]
    t0 = time.time()
    rc, out, err = 0, "", ""
    try:
        p = subprocess.run(cmd, env=env, cwd=os.path.dirname(os.path.abspath(__file__)),
                           capture_output=True, text=True, timeout=args.shmem_probe_timeout)
        rc, out, err = p.returncode, p.stdout, p.stderr
    except subprocess.TimeoutExpired as e:
        rc, err = "timeout", (e.stderr or b"").decode(errors="replace") \
            if isinstance(e.stderr, bytes) else (e.stderr or "")
    except Exception as e:  # noqa: BLE001 - the probe must not cost the headline
        rc, err = "spawn-error", repr(e)
    finally:
        os.unlink(path)
    line = next((ln[len("SHMEM_PROBE "):] for ln in out.splitlines()
                 if ln.startswith("SHMEM_PROBE ")), None)
    mine = {"rank": rank, "exit": rc, "stderr_tail": (err or "")[-400:] if rc != 0 else ""}
    allr = [None] * world
    dist.all_gather_object(allr, mine, group=cpu)
    dist.destroy_process_group(cpu)
    if rank != 0:
        return {}
    bad = [r for r in allr if r["exit"] != 0]
    rec = {"child_wall_s": round(time.time() - t0, 1)}
    if bad or line is None:
        rec["failed"] = bad or [{"rank": 0, "exit": rc, "stderr_tail": "no SHMEM_PROBE line: "
                                 + (err or "")[-300:]}]
        return rec
    try:
        rec.update(json.loads(line))
    except ValueError as e:
        rec["failed"] = [{"rank": 0, "exit": rc, "stderr_tail": f"bad probe line: {e}"}]
    return rec


def _spawn_ranks(n: int) -> int:
    """Run this script under ``torch.distributed.run`` with ``n`` local ranks (loopback
    rendezvous on a free port) as a CHILD process and return its exit status. Called only
    before anything initialised the GPU (no exec from a GPU-initialised process)."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] WORLD_SIZE unset: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr,
          flush=True)
    return subprocess.call(cmd)


def main():
    args = parse()
    from dgraph_amd import Communicator
    from dgraph_amd.utils.config import RunConfig
    from dgraph_amd.utils.metrics import ExperimentLogger

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # not launched by torchrun: start the N ranks ourselves (this process never touches
        # the GPU) and exit with their status — never measure W=1 under an N-GPU label
        sys.exit(_spawn_ranks(args.gpus))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus and not (args.rehearse_world > 1 and world_env == 1):
        print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={world_env} (launch one rank "
              f"per GPU: torchrun --nproc-per-node {args.gpus} bench.py --gpus {args.gpus})",
              file=sys.stderr)
        sys.exit(2)
    if args.link_gbps > 0:
        from dgraph_amd.comm import alltoallv as _a2a

        _a2a.LOOPBACK_LINK_GBPS = args.link_gbps
        if args.link_cus >= 0:
            _a2a.LOOPBACK_CUS = args.link_cus
    cfg = RunConfig.from_env()  # DGRAPH_<SECTION>_<FIELD> overrides (kernel knobs etc.)
    cfg.model.hidden, cfg.model.num_layers, cfg.model.dtype = args.hidden, args.layers, args.dtype
    cfg.data.dataset, cfg.data.global_frac = args.shape, args.global_frac
    cfg.data.scale = args.scale
    args.exec_cfg = cfg.fused  # the fused executor's knobs, resolved once, recorded whole
    comm = Communicator.init_process_group("nccl")
    rank, world = comm.get_rank(), comm.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")
    if dev.type == "cuda":
        cfg.apply()
    dtype = torch.bfloat16 if (args.dtype == "bf16" and dev.type == "cuda") else torch.float32
    mlog = ExperimentLogger(os.path.dirname(args.metrics_jsonl) or ".", args.shape, world) \
        if args.metrics_jsonl else None

    job = Job(args, comm, dev, args.global_frac, dtype)
    log(rank, f"graph built in {job.build_s:.1f}s: V={job.shape.num_nodes} E_msg={job.E_msg} "
              f"halo_rows_total={job.halo_total} train={job.n_train} val={job.n_val} "
              f"test={job.n_test}")
    head_restrict = args.restrict_last
    a2a_plan = getattr(job.graph, "a2a", None)
    # the headline's halo plan (row counts per peer), for the one-sided probe job
    plan_splits = (list(a2a_plan.send_splits), list(a2a_plan.recv_splits)) \
        if (a2a_plan is not None and world > 1 and not job.rehearse) else None
    if dev.type == "cuda":
        torch.cuda.reset_peak_memory_stats()
    ms, final_loss, e_step = timed(job, args.steps, args.warmup, head_restrict, args.verbose)
    peak_gb = torch.cuda.max_memory_allocated() / 1e9 if dev.type == "cuda" else 0.0
    corr = job.correct.clone()
    if world > 1:
        dist.all_reduce(corr)
    val_acc = float(corr[0]) / max(job.n_val, 1)
    test_acc = float(corr[1]) / max(job.n_test, 1)
    halo = job.halo_stats()
    alloc_timed = dict(getattr(job, "alloc_timed", {}))
    mem_setup = getattr(job, "mem_setup_gb", 0.0)
    regions = region_breakdown(job)
    xgmi = link_probe(job) if (world > 1 and not job.rehearse) else {}
    use_fused = job.use_fused
    schedule = job.fused.schedule if job.fused is not None else {}
    pass_for = {str(k): v for k, v in getattr(job.fused, "pass_for", {}).items()} \
        if job.fused is not None else {}
    if job.fused is not None and job.fused.locality is not None:
        pass_for["graph_locality"] = round(job.fused.locality, 4)
    if args.profile_ops:
        _profile_one_step(lambda: job.step(head_restrict), args.profile_ops, rank)
    E_msg, n_train, halo_total = job.E_msg, job.n_train, job.halo_total
    job_recompute = job.recompute
    shape = job.shape
    edges_per_s = args.layers * E_msg / (ms / 1000.0)
    if mlog is not None:
        mlog.metrics(phase="headline", epoch_ms=ms, edges_per_s=edges_per_s,
                     edges_aggregated_per_step=e_step, loss=final_loss, val_acc=val_acc,
                     test_acc=test_acc, peak_hbm_gb=peak_gb, **halo)

    extra = {}
    if not args.no_extra and not job.rehearse:
        ks = max(args.extra_steps, 1)
        if not head_restrict and not use_fused:
            t_ms, _, t_e = timed(job, ks, 1, True)
            extra["train_rows_only"] = {
                "ms_per_step": t_ms, "edges_aggregated_per_step": t_e,
                "note": "output layer aggregated at the train rows only (not a full-graph "
                        "forward; no val/test predictions)"}
        job.free()
        del job
        gc.collect()
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        # structureless secondary: built on every rank; a configuration that does not fit
        # (the fused executor plans its memory and raises before allocating, e.g. fp32 halo
        # rows of a structureless graph at W > 1) is skipped on every rank alike
        try:
            sjob = Job(args, comm, dev, 1.0, dtype)
            ok = 1
        except MemoryError as e:
            sjob, ok = None, 0
            log(rank, f"structureless extra skipped: {e}")
        okt = torch.tensor([ok], dtype=torch.long, device=dev)
        if world > 1:
            dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        if int(okt) == 1:
            try:
                s_ms, s_loss, s_e = timed(sjob, ks, 1, head_restrict)
                extra["structureless"] = {
                    "global_frac": 1.0, "ms_per_step": s_ms,
                    "edges_per_s": args.layers * sjob.E_msg / (s_ms / 1000.0),
                    "edges_aggregated_per_step": s_e, "E_msg": sjob.E_msg,
                    "halo_rows_total": sjob.halo_total, "steps": ks, "warmup": 1,
                    "final_loss": s_loss, **sjob.halo_stats()}
                if sjob.fused is not None:
                    extra["structureless"]["spmm_pass_cols"] = {
                        str(k): v for k, v in sjob.fused.pass_for.items()}
                    if sjob.fused.locality is not None:
                        extra["structureless"]["spmm_pass_cols"]["graph_locality"] = round(
                            sjob.fused.locality, 4)
                    sreg = region_breakdown(sjob)
                    if sreg:
                        extra["structureless"]["regions_ms_max_over_ranks"] = \
                            sreg["ms_max_over_ranks"]
                if mlog is not None:
                    mlog.metrics(phase="structureless", **extra["structureless"])
            except Exception as e:  # noqa: BLE001
                # one GPU: a failed secondary must not cost the headline line (no peers to
                # keep in step); W > 1 re-raises (every rank must take the same path)
                if world > 1:
                    raise
                log(rank, f"structureless extra failed: {e!r}")
                extra["structureless"] = {"global_frac": 1.0, "failed": repr(e)[:300]}
                gc.collect()
                if dev.type == "cuda":
                    torch.cuda.empty_cache()
        else:
            extra["structureless"] = {"global_frac": 1.0, "skipped": "does not fit in HBM at "
                                      "this W (fp32 halo rows of a structureless graph)"}
        if sjob is not None:
            sjob.free()
        del sjob
        if dtype == torch.float32 and dev.type == "cuda" and not args.no_bf16_extra and \
                world == 1:
            # secondary (1 GPU): the same headline graph at bf16 storage/compute (fp32
            # accumulate, fp32 master weights) on the layer-stack path — NOT the reference's
            # precision
            gc.collect()
            torch.cuda.empty_cache()
            import copy

            bargs = copy.copy(args)
            bargs.dtype, bargs.executor = "bf16", "stack"
            bjob = None
            try:  # (one GPU only: a failure here must not cost the headline line)
                bjob = Job(bargs, comm, dev, args.global_frac, torch.bfloat16)
                b_ms, b_loss, b_e = timed(bjob, ks, 1, False)
                extra["bf16_stack"] = {
                    "ms_per_step": b_ms,
                    "edges_per_s": args.layers * bjob.E_msg / (b_ms / 1000.0),
                    "edges_aggregated_per_step": b_e, "steps": ks, "warmup": 1,
                    "final_loss": b_loss,
                    "note": "bf16 storage/compute, fp32 accumulate (below the reference's "
                            "fp32)"}
            except Exception as e:  # noqa: BLE001
                log(rank, f"bf16 extra failed: {e!r}")
                extra["bf16_stack"] = {"failed": repr(e)[:300]}
            if bjob is not None:
                bjob.free()
            del bjob
    else:
        job.free()

    shm = {}
    if plan_splits is not None and not args.no_shmem_probe:
        shm = shmem_probe_child(args, rank, world, plan_splits, dev)
    if args.rehearse_world > 1 and world == 1:
        # not a whole-job number: one rank's compute with a loopback exchange
        print(json.dumps({"rehearsal": True, "rank": args.rehearse_rank,
                          "world": args.rehearse_world,
                          "ms_per_step_compute_loopback": ms, "E_local": E_msg,
                          "halo_rows": halo_total, "peak_mem_gb": round(peak_gb, 2),
                          "mem_after_setup_gb": round(mem_setup, 2),
                          "dtype": args.dtype, "global_frac": args.global_frac,
                          "halo_recompute": job_recompute,
                          "restrict_last": head_restrict,
                          "final_loss_local": final_loss,
                          "executor": "fused" if use_fused else "stack",
                          "link_gbps": args.link_gbps,
                          "link_cus": _link_cus() if args.link_gbps > 0 else 0,
                          "allocator_in_timed_steps": alloc_timed,
                          **({"schedule": schedule} if schedule else {}),
                          **({"halo": halo} if halo else {}),
                          **({"regions": regions} if regions else {})}), flush=True)
    elif rank == 0:
        rec = {
            "metric": "edges_per_s",
            "value": edges_per_s,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "epoch_ms": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.dtype if dev.type == "cuda" else "fp32",
            "executor": "fused (models/sage_fused.py)" if use_fused else "stack (SAGEStackFn)",
            "data": (f"synthetic {shape.name}-shaped graph (V={shape.num_nodes}, "
                     f"directed={shape.num_directed_edges}, symmetrised E_msg={E_msg}, "
                     f"global_frac={args.global_frac}, window={args.window}), random "
                     f"features/labels/splits, random-init weights"),
            "config": {
                "model": f"GraphSAGE-mean {args.layers}-layer hidden {args.hidden}",
                "global_batch": shape.num_nodes,
                "seq_len": None,
                "parallelism": ("single GPU (whole graph, no exchange)" if world == 1 else
                                f"graph-partition{world} (RCCL all-to-all-v halo"
                                + (", layer-1 halo recomputed" if job_recompute else "")
                                + ") + dp-allreduce"),
                "rccl_world_size": (dist.get_world_size() if dist.is_initialized() else 1),
                "process_group_backend": (dist.get_backend() if dist.is_initialized() else None),
                "dataset_shape": shape.name,
                "num_layers": args.layers,
                "hidden": args.hidden,
                "E_msg": E_msg,
                "halo_rows_total": halo_total,
                "train_nodes": n_train,
                "step": ("train-rows-only output layer" if head_restrict else
                         "full-graph forward (all vertices, all layers) + val/test accuracy "
                         "from the same forward + backward + allreduce + Adam"),
                "launch": "HIP graph replay" if args.cuda_graph else "eager",
                "halo_recompute": job_recompute,
                **({"schedule": schedule} if schedule else {}),
                **({"spmm_pass_cols": pass_for} if pass_for else {}),
                "precision": ("bf16 storage/compute, fp32 accumulate, fp32 master weights"
                              if dtype == torch.bfloat16 else
                              "fp32 storage and compute (exact-f32 MFMA GEMMs, fp32 SpMM "
                              "accumulation), fp32 weights: the reference's precision"),
            },
            # SURVEY §5.5 definition, L * E_directed / step (the headline value counts the
            # symmetrised message edges, 2x as many for this undirected graph)
            "edges_per_s_directed": args.layers * shape.num_directed_edges / (ms / 1000.0),
            "E_directed": shape.num_directed_edges,
            "edges_aggregated_per_step": e_step,
            "edges_aggregated_per_s": e_step / (ms / 1000.0),
            "hw_queues": _HWQ_FOUND or "runtime default",
            "final_loss": final_loss,
            "val_acc": val_acc,
            "test_acc": test_acc,
            "peak_mem_gb_rank0": round(peak_gb, 2),
            "mem_after_setup_gb_rank0": round(mem_setup, 2),
            # hipMalloc/hipFree calls and allocation retries inside the timed steps (0 =
            # steady state served from preplanned buffers and the allocator cache)
            "allocator_in_timed_steps": alloc_timed,
            **({"halo": halo} if halo else {}),
            **({"regions": regions} if regions else {}),
            **({"xgmi_probe": xgmi} if xgmi else {}),
            **({"shmem_probe": shm} if shm else {}),
            # every knob the run resolved (RunConfig: comm / kernels / fused executor / model /
            # data), so the line alone reproduces the configuration
            "run_config": cfg.to_dict(),
            **extra,
        }
        print(json.dumps(rec), flush=True)
    comm.destroy()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
