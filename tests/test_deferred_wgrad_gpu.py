"""Weight gradients on the side stream (ops.dense.deferred_wgrad) for the cases the GraphCast
test does not reach: one weight used twice in one call, slices of one weight across calls,
an existing .grad accumulated into, and a parameter that ALSO gets a gradient through
autograd's own accumulation (a non-slice view). A parameter whose every gradient is
deferred equals the inline backward bitwise; the mixed and accumulated cases sum the same
terms in another association (fp32 rounding)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(defer: bool, existing: bool):
    from dgraph_amd.ops.act import linear_act
    from dgraph_amd.ops.dense import deferred_wgrad, linear, linear_sum

    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(3)
    # (scaled like an initialised layer: the activations stay O(1) through the chain)
    W = (torch.randn(128, 256, generator=g) / 16).to(dev).requires_grad_(True)
    V = (torch.randn(128, 128, generator=g) / 11.3).to(dev).requires_grad_(True)
    b = torch.randn(128, generator=g).to(dev).requires_grad_(True)
    x = torch.randn(4096, 128, generator=g).to(dev)
    y = torch.randn(4096, 128, generator=g).to(dev)
    params = (W, V, b)
    if existing:
        for p in params:
            p.grad = torch.full_like(p, 0.5)
    h = linear(x, W[:, :128], b)                       # slice of W
    h = linear_act([(h, W[:, 128:]), (y, V)], None, "silu")  # the other slice, and V
    h = linear_sum([(x, V), (h, V)], None)              # V twice in one call
    h = linear(h, V.t().contiguous().t())              # V behind a non-slice view
    loss = (h * h).mean()
    with deferred_wgrad(defer):
        loss.backward()
    torch.cuda.synchronize()
    return [p.grad.clone() for p in params]


@pytest.mark.parametrize("existing", [False, True])
def test_deferred_wgrad_cases_bitwise(existing):
    from dgraph_amd.ops import dense

    ref = _run(False, existing)
    c0 = dense._DEFER.calls
    got = _run(True, existing)
    assert dense._DEFER.calls > c0
    for a, r, n in zip(got, ref, ("W", "V", "b")):
        if n != "V" and not existing:
            assert torch.equal(a, r), n
        else:  # the same terms in another association: fp32 rounding of the largest term
            torch.testing.assert_close(a, r, atol=1e-5 * float(r.abs().max()), rtol=1e-5)
