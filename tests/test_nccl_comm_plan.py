"""Edge-centric plans (G2): builder fields vs brute force, gather/scatter forward and
backward vs a replicated global ground truth (reference tests/test_NCCLCommPlan.py),
run on gloo process groups at several world sizes."""
import pytest
import torch

from dgraph_amd.plan.nccl_plan import (
    COO_to_NCCLCommPlan,
    COO_to_NCCLEdgeConditionedCommPlan,
    fast_2D_unique,
)


def _coo(world_size, seed=0):
    g = torch.Generator().manual_seed(seed)
    n = 32 * world_size
    adj = torch.rand(n, n, generator=g)
    adj = (adj + adj.t()) / 2
    adj = (adj >= 0.8).float()
    adj.fill_diagonal_(0)
    return n, adj.nonzero().t().contiguous()


def _setup(rank, world):
    n, coo = _coo(world)
    per = (n + world - 1) // world
    offset = torch.arange(world + 1) * per
    offset[-1] = max(int(offset[-1]), n)
    src, dst = coo
    lo, hi = offset[rank], offset[rank + 1]
    local_edges = torch.nonzero((src >= lo) & (src < hi), as_tuple=True)[0]
    return n, coo, offset, local_edges


def _plan_fields(rank, world):
    n, coo, offset, le = _setup(rank, world)
    src, dst = coo
    plan = COO_to_NCCLCommPlan(rank, world, dst, le, offset)
    lo, hi = int(offset[rank]), int(offset[rank + 1])
    my_dst = dst[le]
    internal = (my_dst >= lo) & (my_dst < hi)
    assert torch.equal(plan.local_edge_idx.sort()[0], torch.nonzero(internal, as_tuple=True)[0])
    assert torch.equal(plan.local_vertex_idx.sort()[0], (my_dst[internal] - lo).sort()[0])
    assert torch.equal(plan.boundary_edge_idx.sort()[0], torch.nonzero(~internal, as_tuple=True)[0])
    expect = []
    for r in range(world):
        if r == rank:
            continue
        rs, re = offset[r], offset[r + 1]
        rd = dst[(src >= rs) & (src < re)]
        expect.append(torch.unique(rd[(rd >= lo) & (rd < hi)]))
    exp = torch.cat(expect) if expect else torch.zeros(0, dtype=torch.long)
    assert torch.equal(plan.boundary_vertex_idx.sort()[0], (exp - lo).sort()[0])
    assert sum(plan.boundary_edge_splits) == int(plan.boundary_edge_buffer_map.max() + 1) \
        if plan.boundary_edge_buffer_map.numel() else True
    mu = plan.memory_usage("KB")
    assert mu["total"] > 0 and mu["unit"] == "KB"


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_plan_fields(ranks, world):
    if world == 1:
        _plan_fields(0, 1)
    else:
        ranks(_plan_fields, world)


def _gather_scatter(rank, world, dtype):
    from dgraph_amd import Communicator

    comm = Communicator.init_process_group("nccl")  # gloo underneath on CPU
    try:
        n, coo, offset, le = _setup(rank, world)
        src, dst = coo
        g = torch.Generator().manual_seed(7)
        X = torch.rand(n, 16, generator=g)
        lo, hi = int(offset[rank]), int(offset[rank + 1])
        plan = COO_to_NCCLCommPlan(rank, world, dst, le, offset)
        # gather fwd/bwd
        xl = X[lo:hi].clone().to(dtype).requires_grad_(True)
        E = comm.gather(xl.unsqueeze(0), comm_plan=plan).squeeze(0)
        torch.testing.assert_close(E.float(), X[dst[le]])
        gE = torch.rand(E.shape, generator=g).to(dtype)
        E.backward(gE)
        # ground truth: grad_X[v] = sum over ALL edges e with dst=v of gE_global[e]
        gE_all = torch.zeros(coo.shape[1], 16, dtype=torch.float32)
        # every rank rebuilds the same global gE: seed per edge block
        for r in range(world):
            _, _, _, le_r = _setup(r, world)
            gg = torch.Generator().manual_seed(7)
            torch.rand(n, 16, generator=gg)  # advance identically
            gE_all[le_r] = torch.rand(le_r.numel(), 16, generator=gg)
        gX = torch.zeros(n, 16).index_add_(0, dst, gE_all)
        torch.testing.assert_close(xl.grad.float(), gX[lo:hi], atol=1e-4, rtol=1e-4)
        # scatter fwd/bwd
        el = torch.rand(le.numel(), 16, generator=torch.Generator().manual_seed(3 + rank))
        el = el.to(dtype).requires_grad_(True)
        Y = comm.scatter(el.unsqueeze(0), comm_plan=plan).squeeze(0)
        parts = [None] * world
        for r in range(world):
            _, _, _, le_r = _setup(r, world)
            parts[r] = (le_r, torch.rand(le_r.numel(), 16, generator=torch.Generator().manual_seed(3 + r)))
        Eall = torch.zeros(coo.shape[1], 16)
        for le_r, v in parts:
            Eall[le_r] = v
        Yg = torch.zeros(n, 16).index_add_(0, dst, Eall)
        torch.testing.assert_close(Y.float(), Yg[lo:hi], atol=1e-4, rtol=1e-4)
        gY = torch.ones_like(Y)
        Y.backward(gY)
        torch.testing.assert_close(el.grad.float(), torch.ones(n, 16)[dst[le]])
    finally:
        comm.destroy()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_gather_scatter_fwd_bwd(ranks, world):
    ranks(_gather_scatter, world, torch.float32)


def _edge_conditioned(rank, world):
    n, coo, offset, le = _setup(rank, world)
    src, dst = coo
    ec = COO_to_NCCLEdgeConditionedCommPlan(rank, world, src, dst, le, offset, offset)
    assert ec.source_graph_plan.boundary_edge_idx.numel() == 0
    assert ec.source_graph_plan.local_edge_idx.numel() == le.numel()
    assert ec.dest_graph_plan.num_local_edges == le.numel()
    rev = ec.reverse()
    assert rev.source_graph_plan is ec.dest_graph_plan


def test_edge_conditioned_plan(ranks):
    ranks(_edge_conditioned, 2)


def test_fast_2d_unique_sorted():
    a = torch.tensor([3, 1, 1, 3, 0, 1])
    b = torch.tensor([5, 9, 2, 5, 7, 2])
    ua, ub, inv = fast_2D_unique(a, b)
    assert ua.tolist() == [0, 1, 1, 3] and ub.tolist() == [7, 2, 9, 5]
    assert torch.equal(ua[inv], a) and torch.equal(ub[inv], b)


def test_legacy_alias_kwarg():
    """The reference's own test passed ``global_edges_dst=`` (D6)."""
    n, coo = _coo(1)
    plan = COO_to_NCCLCommPlan(rank=0, world_size=1, global_edges_dst=coo[1],
                               local_edge_list=torch.arange(coo.shape[1]),
                               offset=torch.tensor([0, n]))
    assert plan.boundary_edge_idx.numel() == 0
