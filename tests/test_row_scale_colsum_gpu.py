"""Fused pre-scale + bias-gradient column sums (csrc/kernels/elementwise.hip
row_scale_colsum): the scaled copy equals row_scale_cols bitwise, the column sums match an
fp64 reference and are run-to-run identical; the SAGE backward that uses them reproduces
the separate column-sum pass."""
import pytest
import torch

from dgraph_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("L,F,w,c0", [(100_003, 256, 192, 0), (100_003, 256, 64, 192),
                                      (5, 128, 128, 0), (300_000, 192, 128, 64)])
def test_row_scale_colsum_matches_references(L, F, w, c0):
    from dgraph_amd import _native

    assert _native.load(), "native library missing"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(L + w)
    x = torch.randn(L, F, device=dev, generator=g).to(torch.bfloat16)
    s = torch.rand(L, device=dev, generator=g) + 0.1
    xs = x[:, c0:c0 + w]
    out_a = torch.empty(L, w, device=dev, dtype=torch.bfloat16)
    out_b = torch.empty_like(out_a)
    nb = min(1024, L)
    part = torch.full((nb, F), float("nan"), device=dev)
    K.row_scale_cols(xs, s, out_a)
    K.row_scale_colsum(xs, s, out_b, part[:, c0:c0 + w])
    assert torch.equal(out_a, out_b)
    got = part[:, c0:c0 + w].sum(0)
    ref = xs.double().sum(0).float()
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-2)
    part2 = torch.empty_like(part)
    K.row_scale_colsum(xs, s, out_b, part2[:, c0:c0 + w])
    assert torch.equal(part[:, c0:c0 + w], part2[:, c0:c0 + w])


def test_sage_bias_grad_from_fused_colsum(monkeypatch):
    """bf16 SAGE stack: bias gradients with the fused column sums equal those of the
    separate column-sum pass (same fp32 sums up to summation order)."""
    from dgraph_amd.data.synthetic import SHAPES, build_partition, node_data
    from dgraph_amd.models.sage import GraphSAGE
    from dgraph_amd.parallel import dist_graph
    from dgraph_amd.parallel.dist_graph import DistGraph

    dev = torch.device("cuda", 0)
    shape = SHAPES["ogbn-products"].scaled(0.01)
    p = build_partition(shape, 0, 1, dev)
    csr = p["csr"]
    csr.num_cols = p["L"]
    gr = DistGraph(csr, p["L"], 0, symmetric=True)
    x, y, tr = node_data(shape, 0, p["offsets"], dev, dtype=torch.bfloat16)
    rows = torch.nonzero(tr).squeeze(1)

    def grads():
        torch.manual_seed(0)
        m = GraphSAGE(shape.num_features, 256, shape.num_classes, 3).to(dev)
        out = m(x, gr, out_rows=rows)
        torch.nn.functional.cross_entropy(out.float(), y[rows]).backward()
        return [q.grad.float().clone() for q in m.parameters()]

    fused = grads()
    orig = dist_graph.DistGraph._spmm_col_scaled

    def no_colsum(csr, g, cs, out, scratch, colsum=None):
        return orig(csr, g, cs, out, scratch, None)

    monkeypatch.setattr(dist_graph.DistGraph, "_spmm_col_scaled", staticmethod(no_colsum))
    plain = grads()
    for a, b in zip(fused, plain):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-5)
