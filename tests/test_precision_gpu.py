"""bf16 vs fp32 training parity on the GPU: the fused bf16 GraphSAGE stack (bf16 storage,
MFMA dual GEMMs with fp32 accumulation, bf16 SpMM passes with fp32 accumulation, fp32
master weights and Adam state) follows the fp32 path's loss trajectory.

Both runs start from the same weights on the same scaled ogbn-products-shaped graph and
train the full-graph step of bench.py (all vertices, masked cross-entropy on the train
split) for 30 Adam steps; the bf16 trajectory must stay within a few percent of fp32 at
every step and reach the same loss plateau."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(dtype, steps=30, hidden=256):
    from dgraph_amd.data.synthetic import SHAPES, build_partition, node_data
    from dgraph_amd.models.sage import GraphSAGE
    from dgraph_amd.parallel.dist_graph import DistGraph

    dev = torch.device("cuda", 0)
    shape = SHAPES["ogbn-products"].scaled(0.02)
    p = build_partition(shape, 0, 1, dev)
    csr = p["csr"]
    csr.num_cols = p["L"]
    g = DistGraph(csr, p["L"], 0, symmetric=True)
    x, y, tr = node_data(shape, 0, p["offsets"], dev, dtype=dtype)
    # learnable signal: labels a function of the aggregated features
    with torch.no_grad():
        a = g.aggregate(x.float(), mean=True)
        proj = torch.randn(x.shape[1], shape.num_classes, device=dev,
                           generator=torch.Generator(device=dev).manual_seed(1))
        y = (a @ proj).argmax(1)
    rows = torch.nonzero(tr).squeeze(1)
    torch.manual_seed(0)
    m = GraphSAGE(shape.num_features, hidden, shape.num_classes, 3).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=3e-3)
    losses = []
    for _ in range(steps):
        out = m(x, g, out_rows=rows)
        loss = torch.nn.functional.cross_entropy(out.float(), y[rows])
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses.append(float(loss))
    return torch.tensor(losses)


def test_bf16_fused_stack_tracks_fp32_loss_trajectory():
    from dgraph_amd import _native

    assert _native.load(), "native library missing"
    l32 = _train(torch.float32)
    l16 = _train(torch.bfloat16)
    assert torch.isfinite(l16).all() and torch.isfinite(l32).all()
    assert l32[-1] < 0.8 * l32[0], "fp32 run must learn (sanity)"
    rel = (l16 - l32).abs() / l32
    assert float(rel.max()) < 0.05, rel.tolist()
    assert abs(float(l16[-5:].mean() - l32[-5:].mean())) < 0.03 * float(l32[-5:].mean())
