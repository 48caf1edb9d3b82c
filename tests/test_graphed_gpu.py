"""Whole-step HIP-graph capture (dgraph_amd.utils.graphed) reproduces eager training.

A captured step replays the same kernels on the same memory, so N replayed steps must give
the eager run's losses (and weights) from the same initial state: GraphSAGE on the native
SpMM / MFMA dual-GEMM path (bench.py's full-graph step with val/test counters) and
GraphCast with bf16 compute + fp32 master weights (bench_graphcast.py's step)."""
import pytest
import torch

from dgraph_amd.utils.graphed import GraphedStep, make_capturable


def test_graphed_step_disabled_is_eager():
    calls = []
    gs = GraphedStep(lambda: calls.append(1) or torch.ones(()), enabled=False)
    for _ in range(3):
        gs()
    assert len(calls) == 3 and not gs.captured


def test_make_capturable_sets_groups():
    p = torch.nn.Parameter(torch.randn(4))
    opt = torch.optim.Adam([p], lr=1e-3)
    p.grad = torch.ones(4)
    opt.step()
    make_capturable(opt)
    assert all(g["capturable"] for g in opt.param_groups)
    assert opt.state[p]["step"].dtype == torch.float32


def _sage_run(graphed: bool, steps: int = 6):
    from dgraph_amd.data.synthetic import SHAPES, build_partition, node_data
    from dgraph_amd.models.sage import GraphSAGE
    from dgraph_amd.parallel.dist_graph import DistGraph

    dev = torch.device("cuda", 0)
    shape = SHAPES["ogbn-products"].scaled(0.01)
    p = build_partition(shape, 0, 1, dev)
    csr = p["csr"]
    csr.num_cols = p["L"]
    g = DistGraph(csr, p["L"], 0, symmetric=True)
    x, y, tr = node_data(shape, 0, p["offsets"], dev, dtype=torch.bfloat16)
    rows = torch.nonzero(tr).squeeze(1)
    ev = torch.nonzero(~tr).squeeze(1)
    torch.manual_seed(0)
    m = GraphSAGE(shape.num_features, 256, shape.num_classes, 3).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=3e-3, fused=True)
    make_capturable(opt)  # same optimizer arithmetic in both runs
    hits = torch.zeros((), dtype=torch.long, device=dev)

    def step():
        out, evo = m(x, g, out_rows=rows, eval_rows=ev)
        hits.copy_((evo.argmax(1) == y[ev]).sum())
        loss = torch.nn.functional.cross_entropy(out.float(), y[rows])
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    run = GraphedStep(step, warmup=1) if graphed else step
    losses = []
    for _ in range(steps):
        losses.append(run().detach().clone())
    torch.cuda.synchronize()
    if graphed:
        assert run.captured and run.replays == steps - 1
    return torch.stack(losses).cpu(), [q.detach().float().cpu() for q in m.parameters()], \
        int(hits)


@pytest.mark.gpu
def test_graphed_sage_step_matches_eager():
    from dgraph_amd import _native

    assert _native.load(), "native library missing"
    le, we, he = _sage_run(False)
    lg, wg, hg = _sage_run(True)
    torch.testing.assert_close(lg, le, rtol=1e-5, atol=1e-6)
    for a, b in zip(wg, we):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    assert abs(hg - he) <= max(2, he // 1000)


def _graphcast_run(graphed: bool, steps: int = 5):
    from dgraph_amd import Communicator
    from dgraph_amd.data.graphcast_graph import build_global_graph, partition_graphcast_graph
    from dgraph_amd.data.weather import SyntheticWeatherDataset
    from dgraph_amd.models.graphcast import Config, DGraphCast
    from dgraph_amd.utils.master_weights import MasterWeights

    dev = torch.device("cuda", 0)
    comm = Communicator.init_process_group("nccl")
    try:
        g = build_global_graph(3, (37, 72))
        pg = partition_graphcast_graph(g, 0, 1, group=comm.group).to(dev)
        ds = SyntheticWeatherDataset(pg, 11, 3)
        x, y = (t.to(dev, torch.bfloat16) for t in ds[0])
        cfg = Config()
        cfg.model.hidden_dim = 64
        cfg.model.processor_layers = 3
        cfg.model.input_grid_dim = cfg.model.output_grid_dim = 11
        torch.manual_seed(0)
        model = DGraphCast(cfg, comm).to(dev, torch.bfloat16)
        mw = MasterWeights(model, lambda ps: torch.optim.Adam(ps, lr=1e-3, fused=True))
        make_capturable(mw.optimizer)

        def step():
            model.zero_grad(set_to_none=True)
            out = model(x, pg)
            loss = ((out.float() - y.float()) ** 2).mean()
            loss.backward()
            mw.step()
            return loss

        run = GraphedStep(step, warmup=1) if graphed else step
        losses = [run().detach().clone() for _ in range(steps)]
        torch.cuda.synchronize()
        return torch.stack(losses).cpu(), [p.detach().cpu() for p in mw.master]
    finally:
        comm.destroy()


@pytest.mark.gpu
def test_graphed_graphcast_step_matches_eager():
    from dgraph_amd import _native

    assert _native.load(), "native library missing"
    le, we = _graphcast_run(False)
    lg, wg = _graphcast_run(True)
    torch.testing.assert_close(lg, le, rtol=1e-5, atol=1e-6)
    for a, b in zip(wg, we):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
