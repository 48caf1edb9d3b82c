"""The rehearsal's link model (comm/alltoallv.py LOOPBACK_LINK_GBPS, csrc/comm/symheap.hip
link_delay_kernel) on the GPU:

* the device-side wait holds its stream for the requested wall-clock time;
* a link-delayed loopback exchange is really PENDING when it returns (its copy has not
  landed), and the rows are there after ``wait()`` (a stream-event wait, no host sync);
* one rank of a W-way partition (interior-first, fused fp32 executor) trained behind a slow
  link is BITWISE equal to the same rank with an instant loopback: every consumer of an
  exchange is stream-ordered after it, whatever the transfer time (reference exchange
  regions: experiments/OGB/GCN.py:101-116).
"""
import pytest
import torch

from dgraph_amd import _native
from dgraph_amd.comm import alltoallv as A

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_link_delay_holds_stream():
    _native.load()
    _native.ops().link_delay(10.0, 0)  # first launch loads the code object
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for us in (200.0, 5000.0):
        torch.cuda.synchronize()
        s.record()
        _native.ops().link_delay(us, 0)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e)
        assert us * 1e-3 * 0.95 <= ms <= us * 1e-3 * 1.5 + 0.2, (us, ms)


def test_delayed_loopback_is_pending_then_lands(monkeypatch):
    monkeypatch.setattr(A, "LOOPBACK_LINK_GBPS", 0.05)  # 50 MB/s: ~40 ms for 2 MB
    a2a = A.AllToAllV([1000, 1000], [1000, 1000], None)
    send = torch.randn(2000, 256, device=DEV)
    us = a2a.link_us(256 * 4)
    assert us > 20_000
    recv, work = a2a(send, async_op=True)
    assert not work.is_completed()
    work.wait()  # the current stream now waits for the transfer
    out = recv.clone()
    torch.cuda.synchronize()
    assert work.is_completed()
    assert torch.equal(out, send)


def _rehearsal_step(gbps, steps=2, stream="off"):
    """Rank 0 of a 2-way partition of a scaled papers100M graph, alone (loopback exchange),
    interior-first, on the fused fp32 executor: losses and the last step's gradients."""
    from dgraph_amd.data.synthetic import (SHAPES, SPLIT_TEST, SPLIT_TRAIN, SPLIT_VALID,
                                           build_partition, contiguous_offsets, node_data)
    from dgraph_amd.models.sage import GraphSAGE
    from dgraph_amd.models.sage_fused import FusedSAGE
    from dgraph_amd.parallel.dist_graph import DistGraph
    from dgraph_amd.parallel.reorder import interior_first

    from dgraph_amd.utils.config import ExecutorConfig

    A.LOOPBACK_LINK_GBPS = gbps
    try:
        shape = SHAPES["ogbn-papers100M"].scaled(2e-4)
        part = build_partition(shape, 0, 2, DEV, global_frac=0.05, window=256, rehearse=True)
        csr, send, perm, L_int, loc = interior_first(part["csr"], part["L"],
                                                     part["send_local_idx"])
        assert 0 < L_int < part["L"]
        g = DistGraph(csr, part["L"], part["H"], send, part["send_splits"],
                      part["recv_splits"], None, symmetric=True)
        g.locality_hint = loc
        x, y, split = node_data(shape, 0, contiguous_offsets(shape.num_nodes, 2), DEV,
                                dtype=torch.float32, return_split=True)
        x, y, split = x[perm], y[perm], split[perm]
        tr = torch.nonzero(split == SPLIT_TRAIN).reshape(-1)
        ev = torch.nonzero((split == SPLIT_VALID) | (split == SPLIT_TEST)).reshape(-1)
        torch.manual_seed(0)
        model = GraphSAGE(shape.num_features, 256, shape.num_classes, 3).to(DEV)
        ex = FusedSAGE(model, g, x, tr, y[tr], ev, y[ev], split[ev] == SPLIT_VALID,
                       tr.numel(), chunk_rows=512, release_graph=True,
                       config=ExecutorConfig(halo_stream=stream))
        assert ex.nA >= 1 and ex.stream == (stream == "on")
        losses = []
        for _ in range(steps):
            ex.record = True
            losses.append(ex.step().detach().clone())
            with torch.no_grad():
                for p in model.parameters():
                    p.add_(p.grad, alpha=-0.05)
        reg = ex.region_ms()
        grads = [p.grad.detach().clone() for p in model.parameters()]
        torch.cuda.synchronize()
        return torch.stack(losses), grads, ex.correct.clone(), reg
    finally:
        A.LOOPBACK_LINK_GBPS = 0.0


@pytest.mark.parametrize("stream", ["off", "on"])
def test_rehearsal_delayed_equals_instant_bitwise(stream):
    l0, g0, c0, r0 = _rehearsal_step(0.0, stream=stream)
    # a 0.5 GB/s "link": every exchange (or column block of one) is long
    l1, g1, c1, r1 = _rehearsal_step(0.5, stream=stream)
    assert torch.equal(l0, l1)
    for a, b in zip(g0, g1):
        assert torch.equal(a, b)
    assert torch.equal(c0, c1)
    # the slow link shows up as exposed exchange time, the instant one does not
    ex1 = sum(v for k, v in r1.items() if k.startswith("exchange"))
    ex0 = sum(v for k, v in r0.items() if k.startswith("exchange"))
    assert ex1 > ex0 + 1.0, (r0, r1)


@pytest.mark.parametrize("nbytes", [16, 4096 + 4, 3 * (1 << 20) + 7])
def test_link_copy_bytes_and_hold(nbytes):
    """The link model's transfer kernel copies every byte (16-B vectors and a byte tail)
    and holds its stream for at least the modelled time."""
    _native.load()
    src = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=DEV)
    dst = torch.zeros_like(src)
    _native.ops().link_copy(src, dst, 0.0, 1024, 16)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    dst.zero_()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    _native.ops().link_copy(src, dst, 3000.0, 1024, 16)
    e.record()
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    assert s.elapsed_time(e) >= 3.0 * 0.95
