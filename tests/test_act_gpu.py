"""Fused bias + activation kernels (csrc/kernels/act.hip) and linear_act (ops/act.py) on the
GPU against fp64 / PyTorch references: forward values, dz, the fused bias-gradient column
sums, and the weight / input gradients of one- and two-term products (GraphCast MLPs)."""
import pytest
import torch
import torch.nn.functional as Fn

pytestmark = pytest.mark.gpu

ACT = {0: lambda t: t, 1: Fn.silu, 2: torch.relu}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("F", [128, 73, 256])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_bias_act_kernels(dtype, F, act):
    from dgraph_amd import _native

    ops = _native.ops()
    g = torch.Generator(device="cuda").manual_seed(F + act)
    M = 3001
    z = torch.randn(M, F, device="cuda", generator=g).to(dtype)
    b = torch.randn(F, device="cuda", generator=g)
    dy = torch.randn(M, F, device="cuda", generator=g).to(dtype)
    y = torch.empty_like(z)
    ops.bias_act(z, b, act, y)
    t = (z.double() + b.double()).requires_grad_(True)
    ref = ACT[act](t)
    tol = dict(atol=1e-5, rtol=1e-5) if dtype == torch.float32 else dict(atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(y.double(), ref.detach(), **tol)
    dz = torch.empty_like(z)
    db = ops.bias_act_bwd(dy, z, b, act, dz)
    (gref,) = torch.autograd.grad(ref, t, dy.double())
    torch.testing.assert_close(dz.double(), gref, **tol)
    # the bias gradient sums the stored dz (fp32 accumulation in a fixed order)
    torch.testing.assert_close(db.double(), dz.double().sum(0), atol=1e-3, rtol=1e-5)
    db2 = ops.bias_act_bwd(dy, z, b, act, torch.empty_like(z))
    assert torch.equal(db, db2), "bias gradient must be run-to-run identical"


@pytest.mark.parametrize("two", [False, True])
def test_linear_act_matches_torch(two):
    from dgraph_amd.ops.act import linear_act

    torch.manual_seed(0)
    M, K, N = 4096, 128, 128
    x1 = torch.randn(M, K, device="cuda", requires_grad=True)
    x2 = torch.randn(M, K, device="cuda", requires_grad=True)
    W = torch.randn(N, 2 * K if two else K, device="cuda", requires_grad=True)
    b = torch.randn(N, device="cuda", requires_grad=True)
    terms = [(x1, W[:, :K]), (x2, W[:, K:])] if two else [(x1, W)]
    y = linear_act(terms, b, "silu")
    gy = torch.randn_like(y)
    y.backward(gy)
    got = [t.grad.clone() for t in ((x1, x2, W, b) if two else (x1, W, b))]
    for t in (x1, x2, W, b):
        t.grad = None
    xr = torch.cat([x1, x2], 1) if two else x1
    yr = Fn.silu(Fn.linear(xr.double(), W.double(), b.double()))
    torch.testing.assert_close(y.double(), yr.detach(), atol=1e-4, rtol=1e-4)
    yr.backward(gy.double())
    want = [t.grad for t in ((x1, x2, W, b) if two else (x1, W, b))]
    for a_, w_ in zip(got, want):
        torch.testing.assert_close(a_.double(), w_.double(), atol=5e-3, rtol=1e-4)
