"""GPU tests of the native communication runtime: IPC symmetric heap (remote get / put
kernels, NVSHMEMP2P facade) and the RCCL plan executor.

The symmetric-heap test runs two gloo ranks that share the box's single GPU, so the IPC
mapping, the peer table and the get/put kernels are exercised across real process
boundaries (peer memory on the same device instead of over xGMI). RCCL refuses two ranks
on one device, so the executor is tested at world size 1 (self send/recv).
"""
import pytest
import torch

from conftest import run_ranks

pytestmark = pytest.mark.gpu


def _heap_body(rank, world):
    import torch.distributed as dist

    from dgraph_amd.comm.symheap import NVSHMEMP2P, SymmetricHeap

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    heap = SymmetricHeap(1 << 22, group=None, device=dev)
    assert len(heap.peer_ptrs) == world and heap.owns(heap.local)
    # ---- remote gather: per-rank row counts differ (symmetric slot sized to the max)
    F = 40
    n_rows = [300 + 17 * r for r in range(world)]
    xs = [torch.arange(n * F, dtype=torch.float32).reshape(n, F) + 1e5 * r
          for r, n in enumerate(n_rows)]
    g = torch.Generator().manual_seed(rank)
    E = 1000
    owners = torch.randint(0, world, (E,), generator=g)
    rows = torch.tensor([int(torch.randint(0, n_rows[o], (1,), generator=g)) for o in owners])
    out = heap.remote_gather(xs[rank].to(dev), rows.to(dev), owners.to(dev))
    ref = torch.stack([xs[o][r] for o, r in zip(owners.tolist(), rows.tolist())])
    torch.testing.assert_close(out.cpu(), ref, rtol=0, atol=0)
    # bf16 with a feature width that is not a multiple of 8 (scalar path)
    xb = (xs[rank][:, :13] / 1e3).to(torch.bfloat16).to(dev)
    outb = heap.remote_gather(xb, rows.to(dev), owners.to(dev))
    refb = torch.stack([(xs[o][r, :13] / 1e3).to(torch.bfloat16)
                        for o, r in zip(owners.tolist(), rows.tolist())])
    assert torch.equal(outb.cpu(), refb)
    # ---- put: rank r sends (p + 1) rows to every peer p, landing at row 3 * r
    R = 3 * world
    recv = heap.alloc_tensor((R, F), torch.float32)
    recv.fill_(-1)
    heap.barrier()
    splits = [p + 1 for p in range(world)]
    send = torch.cat([torch.full((p + 1, F), float(100 * rank + p)) for p in range(world)])
    heap.put_rows(send.to(dev), recv, splits, [3 * rank] * world)
    got = recv.cpu()
    for src in range(world):
        k = rank + 1
        torch.testing.assert_close(got[3 * src:3 * src + k],
                                   torch.full((k, F), float(100 * src + rank)))
    # ---- reference-style facade
    NVSHMEMP2P._heap = heap
    assert NVSHMEMP2P.get_rank() == rank and NVSHMEMP2P.get_world_size() == world
    assert NVSHMEMP2P.get_max(rank + 5) == world + 4
    dst = torch.zeros(1, E, F, device=dev)
    NVSHMEMP2P.dist_get(xs[rank].to(dev).unsqueeze(0), dst, rows.to(dev).unsqueeze(0),
                        owners.to(dev).unsqueeze(0), 1, n_rows[rank], F, E)
    torch.testing.assert_close(dst[0].cpu(), ref, rtol=0, atol=0)
    NVSHMEMP2P.finalize()
    dist.barrier()


def test_symmetric_heap_two_processes():
    run_ranks(_heap_body, 2)


def test_symmetric_heap_single_rank():
    from dgraph_amd.comm.symheap import SymmetricHeap

    heap = SymmetricHeap(1 << 20, device=torch.device("cuda", 0))
    x = torch.randn(500, 64, device="cuda").to(torch.bfloat16)
    idx = torch.randint(0, 500, (2000,), device="cuda")
    out = heap.remote_gather(x, idx, torch.zeros_like(idx))
    assert torch.equal(out, x[idx])
    heap.close()


def test_rccl_executor_self_exchange():
    from dgraph_amd.comm.rccl_exec import RCCLExecutor

    ex = RCCLExecutor(None)
    try:
        x = torch.randn(777, 48, device="cuda").to(torch.bfloat16)
        y = torch.empty_like(x)
        ex.alltoallv([x], [y], [777], [777])
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        # async on the executor's stream, consumer waits on the event only
        s = torch.randn(1000, device="cuda")
        r = torch.empty_like(s)
        work = ex.alltoallv([s.view(-1, 1)], [r.view(-1, 1)], [1000], [1000], async_op=True)
        work.wait()
        assert torch.equal((r * 2).cpu(), (s * 2).cpu())
        t = torch.ones(4096, device="cuda")
        ex.all_reduce(t)
        assert float(t.sum()) == 4096.0
    finally:
        ex.close()
