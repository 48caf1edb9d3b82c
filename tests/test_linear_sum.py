"""Fused ``sum_i x_i W_i^T + b (+ acc)`` (ops/dense.py linear_sum, the R-GCN layer
combine): forward and every gradient vs an fp32 PyTorch reference; on the GPU through the
native MFMA dual GEMM (odd term counts chain the running sum through ``cin``)."""
import pytest
import torch

from dgraph_amd.ops.dense import linear_sum


def _case(n_terms, M, K, N, dtype, device, with_acc):
    g = torch.Generator().manual_seed(n_terms * 7 + M)
    xs = [torch.randn(M, K, generator=g).to(device, dtype).requires_grad_(True)
          for _ in range(n_terms)]
    Ws = [(torch.randn(N, K, generator=g) / K ** 0.5).to(device, dtype).requires_grad_(True)
          for _ in range(n_terms)]
    b = torch.randn(N, generator=g).to(device, dtype).requires_grad_(True)
    acc = torch.randn(M, N, generator=g).to(device, dtype).requires_grad_(True) if with_acc else None
    return xs, Ws, b, acc


def _reference(xs, Ws, b, acc, w):
    xs32 = [x.detach().double().requires_grad_(True) for x in xs]
    Ws32 = [W.detach().double().requires_grad_(True) for W in Ws]
    b32 = b.detach().double().requires_grad_(True)
    a32 = None if acc is None else acc.detach().double().requires_grad_(True)
    y = sum(x @ W.t() for x, W in zip(xs32, Ws32)) + b32
    if a32 is not None:
        y = y + a32
    (y * w.double()).sum().backward()
    return y, xs32, Ws32, b32, a32


def _check(n_terms, dtype, device, with_acc, tol):
    M, K, N = 3000, 256, 256
    xs, Ws, b, acc = _case(n_terms, M, K, N, dtype, device, with_acc)
    y = linear_sum(list(zip(xs, Ws)), b, acc)
    w = torch.randn(M, N, device=device, dtype=torch.float32)
    (y.float() * w).sum().backward()
    yr, xr, Wr, br, ar = _reference(xs, Ws, b, acc, w)
    torch.testing.assert_close(y.double(), yr, atol=tol, rtol=tol)
    # gradients: relative Frobenius error (bf16 rounding of g summed over M rows makes
    # near-zero dW entries meaningless elementwise)
    pairs = list(zip(xs + Ws + [b], xr + Wr + [br]))
    if with_acc:
        pairs.append((acc, ar))
    for a, r in pairs:
        err = float((a.grad.double() - r.grad).norm() / r.grad.norm())
        assert err < tol, err


@pytest.mark.parametrize("n_terms,with_acc", [(1, False), (2, True), (3, False), (3, True)])
def test_linear_sum_cpu(n_terms, with_acc):
    _check(n_terms, torch.float64, "cpu", with_acc, 1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("n_terms,with_acc", [(1, False), (2, True), (3, False), (3, True)])
def test_linear_sum_native_bf16_vs_fp64(n_terms, with_acc, monkeypatch):
    from dgraph_amd import _native
    from dgraph_amd.ops import dense

    assert _native.load(), "native library missing"
    calls = []
    orig = dense.dual_gemm
    monkeypatch.setattr(dense, "dual_gemm", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    _check(n_terms, torch.bfloat16, "cuda", with_acc, 1.5e-2)
    # forward: ceil(n/2) chained calls; backward: one dx GEMM per term
    assert len(calls) == (n_terms + 1) // 2 + n_terms
