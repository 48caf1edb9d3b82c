"""GraphCast distributed over TWO PROCESSES on ONE GPU against one process, on the GPU
kernels at fp32: the asynchronous split halo exchange of the encoder / processor / decoder
blocks (parallel/halo.py AsyncHalo: the exchange issued, the edge GEMM and the local
projections run, the wait before the halo rows' projection; the reverse exchange issued
from the halo gradient and waited for at the send rows' gradient) on the one-sided
symmetric-heap transport and on real RCCL (ranks sharing GPU 0 over RCCL's socket
transport), plus a link-delayed loopback
rehearsal of rank 0 of 2 equal to the instant one. Reference: experiments/GraphCast
(distributed GraphCast with the halo exchange of DGraph/distributed/haloExchange.py).
"""
import os

import pytest
import torch

from conftest import run_ranks

pytestmark = pytest.mark.gpu


def _cfg():
    from dgraph_amd.models.graphcast import Config

    cfg = Config()
    cfg.model.hidden_dim = 64
    cfg.model.processor_layers = 2
    cfg.model.input_grid_dim = cfg.model.output_grid_dim = 5
    return cfg


def _run(rank, world, out_dir):
    import torch.distributed as dist

    from dgraph_amd import Communicator
    from dgraph_amd.data.graphcast_graph import build_global_graph, partition_graphcast_graph
    from dgraph_amd.data.weather import SyntheticWeatherDataset
    from dgraph_amd.models.graphcast import DGraphCast
    from dgraph_amd.parallel.grad_sync import GradSync

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = Communicator.init_process_group("nccl")
    try:
        g = build_global_graph(3, (37, 72))
        pg = partition_graphcast_graph(g, rank, world, group=comm.group).to(dev)
        ds = SyntheticWeatherDataset(pg, num_channels=5, num_samples_per_year=3)
        x, y = (t.to(dev) for t in ds[0])
        torch.manual_seed(0)
        model = DGraphCast(_cfg(), comm).to(dev)
        out = model(x, pg)
        n = torch.tensor([float(out.numel())], device=dev)
        if world > 1:
            dist.all_reduce(n)
        loss = ((out - y) ** 2).sum() / n
        loss.backward()
        if world > 1:
            GradSync(model.parameters()).all_reduce()
        gl = loss.detach().clone()
        full = torch.zeros(37 * 72, 5, device=dev)
        full[pg.grid_global_ids.to(dev)] = out.detach()
        if world > 1:
            dist.all_reduce(gl)
            dist.all_reduce(full)
        grads = [p.grad.detach().clone() for p in model.parameters()]
        torch.cuda.synchronize()
        if rank == 0:
            torch.save({"out": full.cpu(), "loss": gl.cpu(), "grads": [t.cpu() for t in grads]},
                       f"{out_dir}/gc_w{world}.pt")
        from dgraph_amd.comm.alltoallv import close_shmem_heaps

        close_shmem_heaps()
    finally:
        comm.destroy()


@pytest.mark.parametrize("transport", ["shmem", "rccl"])
def test_graphcast_two_processes_one_gpu(monkeypatch, tmp_path, transport):
    """shmem: the one-sided symmetric-heap transport over a gloo group; rccl: real RCCL
    (torch ProcessGroupNCCL all-to-all-v, both ranks on GPU 0 over RCCL's socket transport,
    conftest.run_ranks(backend="rccl-one-gpu"))."""
    if transport == "shmem":
        monkeypatch.setenv("DGRAPH_A2A_IMPL", "shmem")
        monkeypatch.setenv("DGRAPH_SYMHEAP_BYTES", str(1 << 28))
        backend = "gloo"
    else:
        monkeypatch.setenv("DGRAPH_A2A_IMPL", "torch")
        backend = "rccl-one-gpu"
    d = str(tmp_path)
    run_ranks(_run, 1, d, timeout=240)
    run_ranks(_run, 2, d, timeout=240, backend=backend)
    r1 = torch.load(f"{d}/gc_w1.pt", weights_only=True)
    r2 = torch.load(f"{d}/gc_w2.pt", weights_only=True)
    torch.testing.assert_close(r2["out"], r1["out"], atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(r2["loss"], r1["loss"], atol=1e-6, rtol=1e-5)
    for a, b in zip(r2["grads"], r1["grads"]):
        rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
        assert rel < 1e-4, rel


def test_graphcast_rehearsal_link_delay_bitwise():
    """Rank 0 of a 2-way partition in this process (patterns built offline, loopback
    exchange): behind a slow modelled link the step is bitwise the instant one — every
    consumer of an asynchronous halo is ordered after it."""
    import dgraph_amd.comm.alltoallv as A
    from dgraph_amd import Communicator
    from dgraph_amd.data.graphcast_graph import build_global_graph, partition_graphcast_graph
    from dgraph_amd.data.weather import SyntheticWeatherDataset
    from dgraph_amd.models.graphcast import DGraphCast

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dev = torch.device("cuda", 0)
    g = build_global_graph(3, (37, 72))
    pg = partition_graphcast_graph(g, 0, 2, rehearse=True).to(dev)
    assert pg.m2m.pattern is not None and pg.g2m.pattern is not None
    ds = SyntheticWeatherDataset(pg, num_channels=5, num_samples_per_year=3)
    x, y = (t.to(dev) for t in ds[0])

    class _Solo:  # a one-process communicator whose engine exchanges by loopback
        def __init__(self):
            from dgraph_amd.comm.nccl_engine import NCCLBackendEngine

            self._engine = NCCLBackendEngine.__new__(NCCLBackendEngine)
            self._engine._group = None

    comm = Communicator.__new__(Communicator)
    comm._engine = _Solo()._engine
    res = []
    try:
        for gbps in (0.0, 0.05):
            A.LOOPBACK_LINK_GBPS = gbps
            torch.manual_seed(0)
            model = DGraphCast(_cfg(), comm).to(dev)
            out = model(x, pg)
            loss = ((out - y) ** 2).mean()
            loss.backward()
            res.append((out.detach().clone(), [p.grad.clone() for p in model.parameters()]))
            torch.cuda.synchronize()
    finally:
        A.LOOPBACK_LINK_GBPS = 0.0
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)


def test_graphcast_deferred_wgrad_bitwise():
    """Weight gradients on the side stream (ops.dense.deferred_wgrad): the same gradients,
    bit for bit, as the inline backward, eagerly and inside a captured HIP graph, and every
    parameter gets one."""
    from dgraph_amd.data.graphcast_graph import build_global_graph, partition_graphcast_graph
    from dgraph_amd.data.weather import SyntheticWeatherDataset
    from dgraph_amd.models.graphcast import DGraphCast
    from dgraph_amd.ops import dense
    from dgraph_amd.utils.graphed import GraphedStep

    dev = torch.device("cuda", 0)
    g = build_global_graph(4, (91, 180))
    pg = partition_graphcast_graph(g, 0, 1).to(dev)
    ds = SyntheticWeatherDataset(pg, num_channels=5, num_samples_per_year=3)
    x, y = (t.to(dev) for t in ds[0])
    torch.manual_seed(0)
    model = DGraphCast(_cfg(), None).to(dev)

    def step(defer):
        model.zero_grad(set_to_none=True)
        loss = ((model(x, pg) - y) ** 2).mean()
        with dense.deferred_wgrad(defer):
            loss.backward()
        return loss

    assert model.branch_streams  # (default) the reference step runs with the branch stream
    step(False)
    ref = [p.grad.clone() for p in model.parameters()]
    c0 = dense._DEFER.calls
    step(True)
    assert dense._DEFER.calls > c0, "no gradient went to the side stream"
    got = [p.grad.clone() for p in model.parameters()]
    for (n, _), a, b in zip(model.named_parameters(), got, ref):
        assert torch.equal(a, b), n
    run = GraphedStep(lambda: step(True), warmup=1)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    assert run.captured
    for (n, p), b in zip(model.named_parameters(), ref):
        assert torch.equal(p.grad, b), n
    # and without the branch stream (the m2g embedding / encoder grid update inline)
    model.branch_streams = False
    step(True)
    torch.cuda.synchronize()
    for (n, p), b in zip(model.named_parameters(), ref):
        assert torch.equal(p.grad, b), n
