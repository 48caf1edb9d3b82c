"""Native synchronised-BatchNorm kernels (csrc/kernels/batchnorm.hip, K-new-7) vs the fp32
PyTorch reference of the same math: statistics, fused normalise/affine/ReLU forward, the
fused backward, odd widths (scalar path), strided rows, a large-mean column (shifted
single-pass statistics must not cancel) and the module-level autograd path."""
import pytest
import torch

from dgraph_amd.models.norm import DistributedBatchNorm1D, _local_moments

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _data(N, F, dtype, seed=0, big_mean=False):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, F, generator=g) * 2.0 + 0.5
    if big_mean:
        x[:, 0] += 1000.0  # |mean| >> std
    return x.to(dtype).to(DEV)


@pytest.mark.parametrize("F", [1, 7, 64, 153, 256, 600])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_moments_match_reference(F, dtype):
    x = _data(5003, F, dtype, seed=F, big_mean=True)
    n, mean, var = _local_moments(x)
    xr = x.float().cpu().double()
    torch.testing.assert_close(mean.cpu().double(), xr.mean(0), atol=1e-4, rtol=1e-5)
    torch.testing.assert_close(var.cpu().double(), xr.var(0, unbiased=False), atol=1e-3,
                               rtol=1e-4)
    assert n == 5003


@pytest.mark.parametrize("F", [7, 153, 256])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu", [False, True])
def test_module_forward_backward(F, dtype, relu):
    torch.manual_seed(0)
    x = _data(4099, F, dtype, seed=F + 1)
    bn = DistributedBatchNorm1D(F).to(DEV)
    with torch.no_grad():
        bn.gamma.uniform_(0.5, 1.5)
        bn.beta.uniform_(-0.5, 0.5)
    xg = x.clone().requires_grad_(True)
    y = bn(xg, relu=relu)
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(3)).to(dtype).to(DEV)
    y.backward(dy)
    # reference: fp32 torch on CPU
    ref = torch.nn.BatchNorm1d(F, eps=bn.eps).double()
    with torch.no_grad():
        ref.weight.copy_(bn.gamma.detach().reshape(-1).double().cpu())
        ref.bias.copy_(bn.beta.detach().reshape(-1).double().cpu())
    xr = x.detach().cpu().double().requires_grad_(True)
    yr = ref(xr)
    if relu:
        yr = torch.relu(yr)
    yr.backward(dy.cpu().double())
    tol = dict(atol=3e-2, rtol=3e-2) if dtype == torch.bfloat16 else dict(atol=2e-4, rtol=2e-4)
    torch.testing.assert_close(y.detach().cpu().double(), yr.detach(), **tol)
    torch.testing.assert_close(xg.grad.cpu().double(), xr.grad, **tol)
    gt = dict(atol=0.5, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=2e-3, rtol=1e-4)
    torch.testing.assert_close(bn.gamma.grad.reshape(-1).cpu().double(), ref.weight.grad, **gt)
    torch.testing.assert_close(bn.beta.grad.reshape(-1).cpu().double(), ref.bias.grad, **gt)


def test_strided_rows_and_determinism():
    from dgraph_amd import _native

    base = _data(3001, 300, torch.bfloat16, seed=5)
    x = base[:, :256]  # row stride 300 (600 B, not 16-B aligned): scalar path
    center = x[0].float().contiguous()
    a = _native.ops().bn_reduce(x, None, center, None, None, None, False, 0)
    b = _native.ops().bn_reduce(x.contiguous(), None, center, None, None, None, False, 0)
    torch.testing.assert_close(a, b, atol=1e-2, rtol=1e-6)  # scalar vs 16-B path order
    c = _native.ops().bn_reduce(x, None, center, None, None, None, False, 0)
    assert torch.equal(a, c)  # fixed-order reduction: bitwise reproducible


def test_empty_rows():
    x = torch.zeros(0, 16, device=DEV, dtype=torch.bfloat16)
    n, mean, var = _local_moments(x)
    assert n == 0 and mean.numel() == 16


@pytest.mark.parametrize("F", [7, 153, 256])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("p", [0.1, 0.5])
def test_fused_dropout_matches_reference(F, dtype, p):
    """BN + ReLU + dropout in the native kernels (mask regenerated from the seed in the
    backward reduce and apply passes) vs an fp64 reference using the same counter-based
    mask (models/norm.dropout_keep_mask): forward values, keep fraction, dx, dgamma, dbeta."""
    from dgraph_amd.models.norm import dropout_keep_mask

    torch.manual_seed(5)
    x = _data(3001, F, dtype, seed=F + 7)
    bn = DistributedBatchNorm1D(F).to(DEV)
    with torch.no_grad():
        bn.gamma.uniform_(0.5, 1.5)
        bn.beta.uniform_(-0.5, 0.5)
    xg = x.clone().requires_grad_(True)
    torch.manual_seed(11)
    y = bn(xg, relu=True, dropout=p)
    torch.manual_seed(11)
    seed = int(torch.randint(0, 1 << 62, (1,), dtype=torch.int64).item())  # the same draw
    keep = dropout_keep_mask(seed, x.shape[0], F, "cpu", p).double()
    frac = float(keep.mean())
    assert abs(frac - (1 - p)) < 0.03, frac
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(3)).to(dtype).to(DEV)
    y.backward(dy)
    ref = torch.nn.BatchNorm1d(F, eps=bn.eps).double()
    with torch.no_grad():
        ref.weight.copy_(bn.gamma.detach().reshape(-1).double().cpu())
        ref.bias.copy_(bn.beta.detach().reshape(-1).double().cpu())
    xr = x.detach().cpu().double().requires_grad_(True)
    yr = torch.relu(ref(xr)) * keep / (1 - p)
    yr.backward(dy.cpu().double())
    tol = dict(atol=6e-2, rtol=3e-2) if dtype == torch.bfloat16 else dict(atol=5e-4, rtol=5e-4)
    torch.testing.assert_close(y.detach().cpu().double(), yr.detach(), **tol)
    torch.testing.assert_close(xg.grad.cpu().double(), xr.grad, **tol)
    torch.testing.assert_close(bn.gamma.grad.reshape(-1).cpu().double(), ref.weight.grad,
                               atol=tol["atol"] * 40, rtol=tol["rtol"])
    torch.testing.assert_close(bn.beta.grad.reshape(-1).cpu().double(), ref.bias.grad,
                               atol=tol["atol"] * 40, rtol=tol["rtol"])
