"""Hub-row split of the transposed segment sums (``IndexMap.transpose_split``): scatter_sum,
the gather adjoint and the edge pre-activation's endpoint gradients give the unsplit result
when a few source rows own most slots (GraphCast's polar mesh vertices)."""
import pytest
import torch
import torch.nn.functional as F

from dgraph_amd.ops import kernels as K
from dgraph_amd.ops.aggregate import gather, scatter_sum
from dgraph_amd.ops.csr import IndexMap
from dgraph_amd.ops.edge_mlp import edge_pre_activation


def _skewed(n_rows, n_slots, seed=0):
    g = torch.Generator().manual_seed(seed)
    idx = torch.randint(0, n_rows, (n_slots,), generator=g)
    idx[: n_slots // 3] = 0  # one hub row with a third of the slots
    idx[n_slots // 3: n_slots // 2] = n_rows - 1
    return idx[torch.randperm(n_slots, generator=g)]


def test_transpose_split_finds_hubs(monkeypatch):
    monkeypatch.setattr(IndexMap, "HUB_CAP", 8)
    im = IndexMap(_skewed(10, 90), 10)
    s = im.transpose_split()
    assert s is not None and set(s.hub_rows.tolist()) >= {0, 9}
    monkeypatch.setattr(IndexMap, "HUB_CAP", 1000)
    assert IndexMap(_skewed(10, 90), 10).transpose_split() is None


def test_scatter_gather_split_gradcheck(monkeypatch):
    monkeypatch.setattr(IndexMap, "HUB_CAP", 4)
    idx = _skewed(7, 60, seed=1)
    im = IndexMap(idx, 7)
    e = torch.randn(60, 3, dtype=torch.float64, requires_grad=True)
    torch.testing.assert_close(scatter_sum(e, im),
                               torch.zeros(7, 3, dtype=torch.float64).index_add_(0, idx, e))
    assert torch.autograd.gradcheck(lambda t: scatter_sum(t, im), (e,))
    x = torch.randn(7, 3, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(lambda t: gather(t, im), (x,))


def test_edge_pre_activation_split_gradcheck(monkeypatch):
    monkeypatch.setattr(IndexMap, "HUB_CAP", 4)
    Vs, Vd, E, H = 6, 5, 50, 3
    src, dst = _skewed(Vs, E, seed=2), _skewed(Vd, E, seed=3)
    Y = torch.randn(E, H, dtype=torch.float64, requires_grad=True)
    P = torch.randn(Vs, H, dtype=torch.float64, requires_grad=True)
    Q = torch.randn(Vd, H, dtype=torch.float64, requires_grad=True)
    sm, dm = IndexMap(src, Vs), IndexMap(dst, Vd)
    fn = lambda y, p, q: edge_pre_activation(y, p, q, sm, dm, "silu")  # noqa: E731
    torch.testing.assert_close(fn(Y, P, Q), F.silu(Y + P[src] + Q[dst]))
    assert torch.autograd.gradcheck(fn, (Y, P, Q))


@pytest.mark.gpu
@pytest.mark.parametrize("Fdim", [64, 128])
def test_scatter_sum_hub_split_gpu(Fdim):
    """Native path at GraphCast's skew (a 6,000-slot row among ~76-slot rows, 128
    features): equal to an fp64 reference, bitwise run to run, and to the unsplit pass."""
    from dgraph_amd import _native

    assert _native.load(), "native library missing"
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    R, per = 40_000, 76
    idx = torch.randint(0, R, (R * per,), generator=g)
    idx[:6000] = 17
    idx[6000:9753] = R - 3
    im = IndexMap(idx.to(dev), R)
    assert im.transpose_split() is not None
    e = torch.randn(idx.numel(), Fdim, generator=g)
    ed = e.to(dev)
    outs = [scatter_sum(ed, im) for _ in range(3)]
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    ref = torch.zeros(R, Fdim, dtype=torch.float64).index_add_(0, idx, e.double())
    torch.testing.assert_close(outs[0].double().cpu(), ref, atol=2e-4, rtol=1e-4)
    t = im.transpose_csr()
    plain = K.spmm(t.rowptr, t.col, ed)
    torch.testing.assert_close(outs[0], plain, atol=2e-4, rtol=1e-5)
    # the adjoint (gather backward) through the same split
    x = torch.randn(R, Fdim, device=dev, requires_grad=True)
    gather(x, im).backward(ed)
    torch.testing.assert_close(x.grad, outs[0], atol=0, rtol=0)
