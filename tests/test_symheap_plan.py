"""The one-sided scatter-add plan (comm/symheap.py ``_ScatterPlan``) on CPU/gloo: the
per-owner pre-aggregation, the slot layout (remote offsets) and the owners' fixed-order
segment sum reproduce a dense scatter-add. The heap's put kernel is emulated by a
two-sided all-to-all-v into the same slot positions (the GPU test in
test_comm_native_gpu.py runs the real put)."""
import pytest
import torch

from conftest import run_ranks


def _body(rank, world, F):
    import torch.distributed as dist

    from dgraph_amd.comm.alltoallv import AllToAllV
    from dgraph_amd.comm.symheap import _ScatterPlan
    from dgraph_amd.ops import kernels as K

    class FakeHeap:
        device = torch.device("cpu")
        group = None

        def __init__(self):
            self.rank, self.world = rank, world

        def alloc_tensor(self, shape, dtype):
            return torch.zeros(shape, dtype=dtype)

    n_out = [30 + 11 * r for r in range(world)]

    def contrib(q):
        g = torch.Generator().manual_seed(7 + q)
        E = 400 + 50 * q
        dr = torch.randint(0, world, (E,), generator=g)
        di = torch.tensor([int(torch.randint(0, n_out[o], (1,), generator=g)) for o in dr])
        return dr, di, torch.randn(E, F, generator=g, dtype=torch.float64)

    dr, di, x = contrib(rank)
    plan = _ScatterPlan(FakeHeap(), di, dr, n_out[rank], F, torch.float64)
    agg = K.spmm(plan.pre.rowptr, plan.pre.col, x)
    # emulate the puts: my block for owner p lands at rows remote_offsets[p] of p's slot
    recv = AllToAllV(plan.send_splits, [0] * world)  # recv splits from the offsets below
    sizes = torch.tensor(plan.send_splits)
    got = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(got, sizes)
    recv_splits = [int(got[q][rank]) for q in range(world)]
    recv = AllToAllV(plan.send_splits, recv_splits)(agg)
    offs = [torch.zeros(world, dtype=torch.long) for _ in range(world)]
    dist.all_gather(offs, torch.tensor(plan.remote_offsets))
    pos = 0
    for q in range(world):
        o = int(offs[q][rank])
        plan.slot[o:o + recv_splits[q]] = recv[pos:pos + recv_splits[q]]
        pos += recv_splits[q]
    out = torch.zeros(n_out[rank], F, dtype=torch.float64)
    post = plan.post
    K.spmm(post.rowptr, post.col, plan.slot, out, beta=1.0, row_map=post.row_map)
    ref = torch.zeros(n_out[rank], F, dtype=torch.float64)
    for q in range(world):
        rq, iq, vq = contrib(q)
        m = rq == rank
        ref.index_add_(0, iq[m], vq[m])
    torch.testing.assert_close(out, ref, atol=1e-10, rtol=1e-10)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_scatter_plan_matches_dense(world):
    run_ranks(_body, world, 5)
