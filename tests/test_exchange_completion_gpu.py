"""Completion contract of every AllToAllV transport (comm/alltoallv.py): a work's
``wait()`` orders the WAITING stream after all device work the call enqueued, on any
stream — also when the call is issued from the comm side stream, as the overlap schedules
of the fused executor do (sage_fused.py ``_exchange`` / ``_on_comm_stream``).

The hazard is forced deterministically: a long ``link_delay`` kernel is enqueued on the
side stream BEFORE an instant-loopback exchange issued there, so the exchange's copy cannot
have run when the compute stream consumes the receive buffer unless the compute stream
really waits for it. Round 4 returned a no-op work here (the driver's bitwise failure,
VERDICT r4 Weak 1). Reference contract: ``put`` is synchronous
(DGraph/distributed/Engine.py:67-86); the halo buffer is consumed after it returns
(haloExchange.py:47-62).
"""
import pytest
import torch

from dgraph_amd import _native
from dgraph_amd.comm import alltoallv as A

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _delay_side(us: float):
    side = A._side_stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        _native.ops().link_delay(float(us), 0)
    return side


def test_side_stream_loopback_orders_consumer():
    _native.load()
    A_GBPS = A.LOOPBACK_LINK_GBPS
    A.LOOPBACK_LINK_GBPS = 0.0  # the instant loopback (the racy path of round 4)
    try:
        a2a = A.AllToAllV([3000, 3000], [3000, 3000], None)
        send = torch.randn(6000, 128, device=DEV)
        out = torch.zeros_like(send)
        torch.cuda.synchronize()
        side = _delay_side(30_000.0)  # 30 ms
        with torch.cuda.stream(side):
            recv, work = a2a(send, out=out, async_op=True)
        work.wait()  # compute stream
        got = recv.clone()  # consumer on the compute stream
        torch.cuda.synchronize()
        assert torch.equal(got, send)
    finally:
        A.LOOPBACK_LINK_GBPS = A_GBPS


def test_side_stream_reverse_loopback_orders_consumer():
    """The reverse direction (a2a_rev of the streamed B1b exchange): more received rows
    than sent (the rest read as zero), consumed by an accumulate on the compute stream."""
    _native.load()
    a2a = A.AllToAllV([1000, 1000], [1500, 1500], None)
    send = torch.randn(2000, 64, device=DEV)
    out = torch.full((3000, 64), 7.0, device=DEV)
    acc = torch.ones(3000, 64, device=DEV)
    torch.cuda.synchronize()
    side = _delay_side(30_000.0)
    with torch.cuda.stream(side):
        recv, work = a2a(send, out=out, async_op=True)
    work.wait()
    acc.add_(recv)
    torch.cuda.synchronize()
    ref = torch.ones(3000, 64, device=DEV)
    ref[:2000] += send
    assert torch.equal(acc, ref)


def _streamed_step(delay_us: float, stream: str, steps: int = 2):
    """Rank 0 of a 2-way partition on the fused fp32 executor with an INSTANT loopback
    whose every exchange is preceded on the issuing stream by a ``delay_us`` kernel."""
    from test_linkdelay_gpu import _rehearsal_step  # tests/ is on sys.path (rootdir-less import)

    orig = A.AllToAllV.__call__

    def delayed(self, send, out=None, async_op=False):
        if delay_us > 0:
            _native.ops().link_delay(float(delay_us), 0)
        return orig(self, send, out=out, async_op=async_op)

    A.AllToAllV.__call__ = delayed
    try:
        return _rehearsal_step(0.0, steps=steps, stream=stream)
    finally:
        A.AllToAllV.__call__ = orig


@pytest.mark.parametrize("stream", ["off", "on"])
def test_delayed_instant_exchanges_bitwise(stream):
    """Every exchange of the fused executor (layer halos, streamed column blocks forward
    and reverse) made slow on its own stream: results bitwise equal to the undelayed run."""
    l0, g0, c0, _ = _streamed_step(0.0, stream)
    l1, g1, c1, _ = _streamed_step(3000.0, stream)
    assert torch.equal(l0, l1)
    for a, b in zip(g0, g1):
        assert torch.equal(a, b)
    assert torch.equal(c0, c1)
