#!/usr/bin/env python3
"""GraphCast training-step and MeshEdgeBlock micro-benchmark
(experiments/GraphCast/microbenchmark_graphcast.py behaviour).

* ``--mode step``: full DGraphCast forward + backward + Adam on the 721 x 1440 grid with
  the level-6 multimesh (1.04 M grid nodes, 40 962 mesh nodes, 327 660 mesh edges,
  ~1.6 M grid2mesh and 3.1 M mesh2grid edges); reports ms/step and edge updates/s.
* ``--mode edge``: one processor MeshEdgeBlock (halo exchange + fused edge MLP) at
  ``--hidden`` (reference: F=512), timing the communication and compute parts separately
  with HIP events.

Runs single-process or under torchrun (latitude-band graph partition, RCCL halos); rank 0
prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="step", choices=["step", "edge"])
    ap.add_argument("--mesh-level", type=int, default=6)
    ap.add_argument("--grid", default="721x1440")
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--channels", type=int, default=None,
                    help="grid channels (default: by --channel-config)")
    ap.add_argument("--channel-config", default="reference-73",
                    choices=["reference-73", "era5-37"],
                    help="reference-73: the reference's 73 climate channels "
                         "(graphcast_config.py:42); era5-37: ERA5 on 37 pressure levels, "
                         "6 atmospheric variables x 37 + 5 surface = 227 channels "
                         "(BASELINE config 5)")
    ap.add_argument("--profile-ops", default="",
                    help="torch.profiler per-op device-time table of one step -> PATH")
    ap.add_argument("--dtype", default="fp32", choices=["bf16", "fp32"],
                    help="fp32 (default) = the reference's precision (experiments/GraphCast has no "
                         "casts); bf16 = bf16 compute with fp32 master weights")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cuda-graph", action="store_true",
                    help="--mode step: capture the whole step into a HIP graph after one "
                         "eager step and replay it (dgraph_amd.utils.graphed)")
    ap.add_argument("--mesh-vertex-placement", default=None,
                    help="mesh_vertex_rank_placement.pt (int [V_mesh] ranks, loaded "
                         "weights_only); default: latitude bands")
    ap.add_argument("--dedup-mesh-edges", action="store_true",
                    help="one processor edge per multimesh edge pair (327 660 at level 6); "
                         "default: the reference's graph, every multimesh edge carried twice "
                         "(655 320, experiments/GraphCast/tests/test_single_graph_data.py)")
    ap.add_argument("--partition", default="latitude", choices=["latitude", "aligned"],
                    help="latitude: equal grid-row bands, mesh by latitude quantiles; aligned: "
                         "one set of cost-balanced latitude cuts for grid and mesh (small halos)")
    ap.add_argument("--branch-streams", type=int, default=1, choices=[0, 1],
                    help="1: independent parts of the step on a second stream")
    ap.add_argument("--wgrad-stream", type=int, default=1, choices=[0, 1],
                    help="1: weight gradients on a side stream (ops.dense.deferred_wgrad)")
    ap.add_argument("--rehearse-world", type=int, default=0,
                    help="single process: rank --rehearse-rank of a W-way partition, every "
                         "halo exchange a loopback (patterns of all ranks built in memory)")
    ap.add_argument("--rehearse-rank", type=int, default=0)
    ap.add_argument("--link-gbps", type=float, default=0.0,
                    help="rehearsal link model: each loopback exchange takes latency + "
                         "largest per-peer message / GBPS (comm/alltoallv.py)")
    ap.add_argument("--regions", action="store_true",
                    help="after the timed steps, one more step with per-region device times "
                         "(exchange-wait = exposed halo exchange), as the reference's "
                         "microbenchmark times communication vs processing")
    a = ap.parse_args()
    if a.link_gbps > 0:
        import dgraph_amd.comm.alltoallv as _A

        _A.LOOPBACK_LINK_GBPS = a.link_gbps
    if a.channels is None:
        a.channels = 73 if a.channel_config == "reference-73" else 6 * 37 + 5

    import torch.distributed as dist

    from dgraph_amd import Communicator
    from dgraph_amd.data.graphcast_graph import build_global_graph, partition_graphcast_graph
    from dgraph_amd.ops.dense import deferred_wgrad
    from dgraph_amd.data.weather import SyntheticWeatherDataset
    from dgraph_amd.models.graphcast import Config, DGraphCast, MeshEdgeBlock
    from dgraph_amd.parallel.grad_sync import GradSync

    comm = Communicator.init_process_group("nccl")
    rank, W = comm.get_rank(), comm.get_world_size()
    rehearse = a.rehearse_world > 1 and W == 1
    p_rank, p_world = (a.rehearse_rank, a.rehearse_world) if rehearse else (rank, W)
    dev = torch.device("cuda", torch.cuda.current_device())
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    t0 = time.perf_counter()
    g = build_global_graph(a.mesh_level, tuple(int(v) for v in a.grid.split("x")),
                           duplicate_mesh_edges=not a.dedup_mesh_edges)
    mesh_part = None
    if a.mesh_vertex_placement:
        from dgraph_amd.data.graphcast_graph import load_mesh_placement

        mesh_part = load_mesh_placement(a.mesh_vertex_placement, g.mesh_xyz.shape[0], p_world)
    pg = partition_graphcast_graph(g, p_rank, p_world, mesh_part=mesh_part, group=comm.group,
                                   rehearse=rehearse, partition=a.partition).to(dev)
    build_s = time.perf_counter() - t0
    cfg = Config()
    cfg.model.hidden_dim = a.hidden
    cfg.model.processor_layers = a.layers
    cfg.model.input_grid_dim = cfg.model.output_grid_dim = a.channels
    torch.manual_seed(0)

    def sync():
        torch.cuda.synchronize()
        if W > 1:
            dist.barrier()

    result = {}
    if a.mode == "step":
        ds = SyntheticWeatherDataset(pg, a.channels, 3)
        x, y = (t.to(dev, dt) for t in ds[0])
        model = DGraphCast(cfg, comm).to(dev, dt)
        model.branch_streams = bool(a.branch_streams)
        gs = GradSync(model.parameters())
        if dt == torch.float32:
            opt = torch.optim.Adam(model.parameters(), lr=1e-4, fused=True)
            masters = None
        else:
            # bf16 compute, fp32 master weights + Adam state (the trainer's scheme)
            from dgraph_amd.utils.master_weights import MasterWeights

            masters = MasterWeights(model, lambda ps: torch.optim.Adam(ps, lr=1e-4, fused=True))
            opt = masters.optimizer

        def step():
            model.zero_grad(set_to_none=True)
            out = model(x, pg)
            loss = ((out.float() - y.float()) ** 2).mean()
            with deferred_wgrad(bool(a.wgrad_stream)):
                loss.backward()
            gs.all_reduce()
            if masters is not None:
                masters.step()
            else:
                opt.step()
            return loss

        run = step
        if a.cuda_graph:
            from dgraph_amd.utils.graphed import GraphedStep, make_capturable

            make_capturable(opt)
            run = GraphedStep(step, warmup=1)
        for _ in range(a.warmup):
            run()
        sync()
        t = time.perf_counter()
        for _ in range(a.steps):
            loss = run()
        sync()
        ms = (time.perf_counter() - t) * 1e3 / a.steps
        edges = a.layers * g.m2m[0].size + g.g2m[0].size + g.m2g[0].size
        if a.profile_ops and rank == 0:
            from torch.profiler import ProfilerActivity, profile

            with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                         record_shapes=True) as prof:
                step()
                sync()
            with open(a.profile_ops, "w") as f:
                f.write(prof.key_averages(group_by_input_shape=True).table(
                    sort_by="self_cuda_time_total", row_limit=40, max_name_column_width=60,
                    max_shapes_column_width=80))
                # the same step attributed to aten ops (which op launched each elementwise
                # kernel), heaviest first
                rows = [e for e in prof.key_averages(group_by_input_shape=True)
                        if e.key.startswith("aten::") or e.key.startswith("dgraph_amd::")]
                rows.sort(key=lambda e: -e.self_device_time_total)
                f.write("\n\nop-level (self device us, calls, shapes):\n")
                for e in rows[:80]:
                    f.write(f"{e.self_device_time_total:10.0f} {e.count:5d}  {e.key:36s} "
                            f"{str(e.input_shapes)[:110]}\n")
        regions = {}
        if a.regions or rehearse:
            from dgraph_amd.utils.timing import TimingReport

            TimingReport.reset()
            TimingReport.init()
            for _ in range(2):
                step()
            # per-step totals of each region over the second step (a region may occur
            # several times per step: one exchange-wait per halo exchange)
            for k, lst in TimingReport.resolve().items():
                vals = [v for v in lst if isinstance(v, float)]
                regions[k] = round(sum(vals[len(vals) // 2:]), 3)
            TimingReport.reset()
        halo_rows = {k: int(es.pattern.num_halo_vertices) if es.pattern is not None else 0
                     for k, es in (("m2m", pg.m2m), ("g2m", pg.g2m), ("m2g", pg.m2g))}
        result = {"metric": "graphcast_step_ms", "ms_per_step": ms,
                  "regions_ms": regions, "halo_rows": halo_rows,
                  "local_grid": int(pg.num_local_grid), "local_mesh": int(pg.num_local_mesh),
                  **({"rehearsal": {"world": p_world, "rank": p_rank,
                                    "link_gbps": a.link_gbps}} if rehearse else {}),
                  "channels": a.channels, "channel_config": a.channel_config,
                  "partition": a.partition if not a.mesh_vertex_placement else "placement file",
                  "mesh_edges": int(g.m2m[0].size), "duplicate_mesh_edges":
                  not a.dedup_mesh_edges,
                  "launch": "HIP graph replay" if a.cuda_graph else "eager",
                  "wgrad_stream": bool(a.wgrad_stream),
                  "branch_streams": bool(a.branch_streams),
                  "precision": "bf16 compute, fp32 master weights" if masters is not None
                  else "fp32",
                  "edge_updates_per_s": edges / (ms / 1e3), "loss": float(loss),
                  "peak_mem_gb": torch.cuda.max_memory_allocated() / 1e9}
    else:
        H = a.hidden
        blk = MeshEdgeBlock(H, H, H, H, comm, H).to(dev, dt)
        n = torch.randn(pg.num_local_mesh, H, device=dev, dtype=dt)
        e = torch.randn(pg.m2m.num_edges, H, device=dev, dtype=dt)
        from dgraph_amd.parallel.halo import HaloExchange

        hx = HaloExchange(comm)
        comm_ms, comp_ms = [], []
        for it in range(a.warmup + a.steps):
            s0, s1, s2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            s0.record()
            n_all = torch.cat([n, hx(n, pg.m2m.pattern)]) if pg.m2m.pattern is not None else n
            s1.record()
            out = blk.fused(n, n_all, e, pg.m2m.agg_map(), pg.m2m.other_map())
            s2.record()
            torch.cuda.synchronize()
            if it >= a.warmup:
                comm_ms.append(s0.elapsed_time(s1))
                comp_ms.append(s1.elapsed_time(s2))
        del out
        result = {"metric": "mesh_edge_block_ms", "comm_ms": sum(comm_ms) / len(comm_ms),
                  "compute_ms": sum(comp_ms) / len(comp_ms), "edges": pg.m2m.num_edges}
    t = torch.tensor([result.get("ms_per_step", result.get("compute_ms", 0.0))], device=dev)
    if W > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        result.update({"n_gpus": W, "dtype": a.dtype, "hidden": a.hidden, "layers": a.layers,
                       "grid": a.grid, "mesh_level": a.mesh_level, "graph_build_s": build_s,
                       "max_over_ranks_ms": float(t)})
        print(json.dumps(result), flush=True)
    comm.destroy()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
