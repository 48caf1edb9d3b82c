"""Index-based API (G1) on every backend engine, with the reference's literal graphs
(tests/test_nccl_backend.py:21-232, test_mpi_backend.py:20-198,
test_nvshmem_backend.py:100-200) — on gloo process groups (W=2). The reference's NCCL
G1 path raised NameError (D1); here all three engines agree, with and without caches."""
import pytest
import torch


def _nccl_gather(rank, world):
    from dgraph_amd import Communicator

    comm = Communicator.init_process_group("nccl")
    try:
        torch.manual_seed(0)
        X = torch.randn(1, 4, 2)
        coo = torch.tensor([[0, 0, 0, 1, 2, 2, 2, 3], [1, 2, 3, 0, 3, 0, 3, 0]])
        rm = torch.tensor([[0, 0, 0, 0, 1, 1, 1, 1], [0, 1, 1, 0, 1, 0, 1, 0]])
        out_all = torch.stack([X[0, coo[k]] for k in range(2)])
        xl = comm.get_local_rank_slice(X)
        assert xl.shape == (1, 2, 2)
        for i in range(2):
            m = torch.stack([rm[0], rm[i]])
            got = comm.gather(xl, coo[[i]], m)
            assert got.shape == (1, 4, 2)
            torch.testing.assert_close(got[0], out_all[i, 4 * rank:4 * rank + 4])
    finally:
        comm.destroy()


def _nccl_gather_unbalanced(rank, world):
    from dgraph_amd import Communicator

    comm = Communicator.init_process_group("nccl")
    try:
        torch.manual_seed(0)
        X = torch.randn(1, 8, 2)
        placement = torch.tensor([0, 0, 0, 0, 1, 1, 1, 1])
        coo = torch.tensor([[0, 1], [0, 2], [0, 3], [1, 0], [1, 2], [1, 3], [2, 0], [2, 1],
                            [2, 3], [2, 5], [3, 0], [3, 1], [3, 2], [3, 4], [4, 3], [4, 5],
                            [4, 6], [5, 2], [5, 4], [5, 7], [6, 4], [6, 7], [7, 5], [7, 6]]).T
        rm = (coo > 3).long()
        xl = comm.get_local_rank_slice(X)
        assert torch.equal(xl, X[:, placement == rank])
        for i in range(2):
            m = torch.stack([rm[0], rm[i]])
            got = comm.gather(xl, coo[[i]], m)
            exp = X[0, coo[i]][rm[0] == rank]
            torch.testing.assert_close(got[0], exp)
    finally:
        comm.destroy()


def _nccl_scatter(rank, world, use_cache):
    from dgraph_amd import Communicator
    from dgraph_amd.plan.legacy_cache import NCCLScatterCacheGenerator

    comm = Communicator.init_process_group("nccl")
    try:
        torch.manual_seed(0)
        X = torch.randn(1, 8, 4)
        idx = torch.tensor([[0, 0, 0, 1, 2, 2, 2, 3], [1, 2, 3, 0, 3, 0, 3, 0]])
        rm = torch.tensor([[0, 0, 0, 0, 1, 1, 1, 1], [0, 1, 1, 0, 1, 0, 1, 0]])
        xl = comm.get_local_tensor(X, rm[0], dim=1)
        for i in range(2):
            exp = torch.zeros(4, 4).index_add_(0, idx[i], X[0])
            m = torch.stack([rm[0], rm[i]])
            if use_cache:
                cache = NCCLScatterCacheGenerator(idx[i], rm[0], rm[i], 2, rank, world)
                got = comm.scatter(xl, cache=cache)
            else:
                got = comm.scatter(xl, idx[i], m, 2)
            assert got.shape == (1, 2, 4)
            torch.testing.assert_close(got[0], exp[2 * rank:2 * rank + 2])
    finally:
        comm.destroy()


def _nccl_gather_cache_backward(rank, world):
    from dgraph_amd import Communicator
    from dgraph_amd.plan.legacy_cache import NCCLGatherCacheGenerator

    comm = Communicator.init_process_group("nccl")
    try:
        torch.manual_seed(0)
        X = torch.randn(1, 4, 3)
        coo = torch.tensor([[0, 0, 0, 1, 2, 2, 2, 3], [1, 2, 3, 0, 3, 0, 3, 0]])
        rm = torch.tensor([[0, 0, 0, 0, 1, 1, 1, 1], [0, 1, 1, 0, 1, 0, 1, 0]])
        for i in range(2):
            xl = comm.get_local_rank_slice(X).clone().requires_grad_(True)
            cache = NCCLGatherCacheGenerator(coo[i], rm[0], rm[i], 2, rank, world)
            got = comm.gather(xl, cache=cache)
            torch.testing.assert_close(got[0], X[0, coo[i]][4 * rank:4 * rank + 4])
            got.sum().backward()
            cnt = torch.bincount(coo[i], minlength=4).float()
            torch.testing.assert_close(xl.grad[0], cnt[2 * rank:2 * rank + 2, None].expand(2, 3))
    finally:
        comm.destroy()


def _mpi(rank, world):
    from dgraph_amd import Communicator

    comm = Communicator.init_process_group("mpi", SKIP_NCCL_ASSERT=True)
    try:
        torch.manual_seed(0)
        X = torch.randn(1, 4, 64)
        coo = torch.tensor([[0, 0, 0, 1, 1, 2, 2, 3], [1, 2, 3, 0, 3, 0, 3, 0]])
        rm = torch.tensor([[0, 0, 0, 0, 0, 1, 1, 1], [0, 1, 1, 0, 1, 0, 1, 0]])
        xl = comm.get_local_rank_slice(X, dim=1)
        li = comm.get_local_rank_slice(coo.unsqueeze(0))
        lm = comm.get_local_rank_slice(rm.unsqueeze(0))
        torch.testing.assert_close(xl, X[:, 2 * rank:2 * rank + 2])
        for i in range(2):
            got = comm.gather(xl, li[:, i], lm[0][[i], :])
            torch.testing.assert_close(got, X[:, coo[i]][:, 4 * rank:4 * rank + 4])
        # scatter
        torch.manual_seed(0)
        Xs = torch.randn(1, 8, 4)
        for i in range(2):
            lis = comm.get_local_rank_slice(coo[[i]], dim=1)
            lms = comm.get_local_rank_slice(rm[[i]], dim=1)
            xs = comm.get_local_rank_slice(Xs, dim=1)
            got = comm.scatter(xs, lis, 2, lms)
            exp = torch.zeros(4, 4).index_add_(0, coo[i], Xs[0])
            torch.testing.assert_close(got[0], exp[2 * rank:2 * rank + 2])
        # put (implemented, D2)
        send = torch.full((2, 3), float(rank))
        recv = torch.empty(2, 3)
        off = torch.tensor([0, 1, 2])
        comm.put(send, recv, off, off)
        assert recv[:, 0].tolist() == [0.0, 1.0]
        comm.barrier()
    finally:
        comm.destroy()


def _shmem(rank, world):
    from dgraph_amd import Communicator

    comm = Communicator.init_process_group("nvshmem")
    try:
        torch.manual_seed(0)
        X = torch.randn(1, 4, 8)
        coo = torch.tensor([[0, 0, 0, 1, 1, 2, 2, 3], [1, 2, 3, 0, 3, 0, 3, 0]])
        rm = torch.tensor([[0, 0, 0, 0, 0, 1, 1, 1], [0, 1, 1, 0, 1, 0, 1, 0]])
        for i in range(2):
            li = comm.get_local_rank_slice(coo[[i]], dim=1)
            lm = comm.get_local_rank_slice(rm[[i]], dim=1)
            xl = comm.get_local_rank_slice(X, dim=1)
            got = comm.gather(xl, li, lm)
            torch.testing.assert_close(got, X[:, coo[i]][:, 4 * rank:4 * rank + 4])
            xs = comm.get_local_rank_slice(torch.randn(1, 8, 8, generator=torch.Generator().manual_seed(i)), dim=1)
            got = comm.scatter(xs, li, lm, 2)
            full = torch.randn(1, 8, 8, generator=torch.Generator().manual_seed(i))
            exp = torch.zeros(4, 8).index_add_(0, coo[i], full[0])
            torch.testing.assert_close(got[0], exp[2 * rank:2 * rank + 2])
        assert comm.engine.get_max(rank + 3) == world + 2
    finally:
        comm.destroy()


def test_nccl_g1_gather(ranks):
    ranks(_nccl_gather, 2)


def test_nccl_g1_gather_unbalanced(ranks):
    ranks(_nccl_gather_unbalanced, 2)


@pytest.mark.parametrize("use_cache", [False, True])
def test_nccl_g1_scatter(ranks, use_cache):
    ranks(_nccl_scatter, 2, use_cache)


def test_nccl_g1_gather_cache_backward(ranks):
    ranks(_nccl_gather_cache_backward, 2)


def test_mpi_backend(ranks):
    ranks(_mpi, 2)


def test_shmem_backend_two_sided_transport(ranks):
    ranks(_shmem, 2)


def test_offline_cache_matches_collective_lowering(ranks, tmp_path):
    """Offline (no-communication) cache generation == the collective builder."""
    ranks(_offline_vs_collective, 3)


def _offline_vs_collective(rank, world):
    from dgraph_amd.parallel.index_ops import lower_local_form
    from dgraph_amd.plan.legacy_cache import NCCLGatherCacheGenerator, load_cache, save_cache
    import tempfile, os

    g = torch.Generator().manual_seed(5)
    n_per = 6
    E = 40
    idx = torch.randint(0, n_per * world, (E,), generator=g)
    place = torch.randint(0, world, (E,), generator=g)
    owner = idx // n_per
    cache = NCCLGatherCacheGenerator(idx, place, owner, n_per, rank, world)
    mine = place == rank
    plan = lower_local_form(idx[mine], owner[mine], n_per, rank, world)
    for f in ("local_edge_idx", "local_vertex_idx", "boundary_edge_idx",
              "boundary_edge_buffer_map", "boundary_vertex_idx"):
        assert torch.equal(getattr(cache.plan, f).long(), getattr(plan, f).long()), f
    assert cache.plan.boundary_edge_splits == plan.boundary_edge_splits
    assert cache.plan.boundary_vertex_splits == plan.boundary_vertex_splits
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "c.pt")
        save_cache(cache, p)
        c2 = load_cache(p)
        assert torch.equal(c2.plan.boundary_vertex_idx, cache.plan.boundary_vertex_idx)


def _legacy_fns(rank, world):
    import torch.distributed as dist

    from dgraph_amd.comm.alltoallv import _nccl_alltoallv_with_dict, torch_alltoallv_with_comm_map
    from dgraph_amd.parallel.index_ops import GatherFunction, ScatterFunction

    dist_ok = dist.is_initialized()
    assert dist_ok
    torch.manual_seed(0)
    X = torch.randn(1, 4, 2)
    coo = torch.tensor([[0, 0, 0, 1, 2, 2, 2, 3], [1, 2, 3, 0, 3, 0, 3, 0]])
    rm = torch.tensor([[0, 0, 0, 0, 1, 1, 1, 1], [0, 1, 1, 0, 1, 0, 1, 0]])
    xl = X[:, 2 * rank:2 * rank + 2].clone().requires_grad_(True)
    got = GatherFunction.apply(xl, coo[[1]], rm[0], rm[1], rank, world)
    torch.testing.assert_close(got[0], X[0, coo[1]][rm[0] == rank])
    got.sum().backward()
    deg = torch.bincount(coo[1], minlength=4).float()
    torch.testing.assert_close(xl.grad[0], deg[2 * rank:2 * rank + 2].unsqueeze(1).expand(2, 2))
    Y = torch.arange(16.0).reshape(1, 8, 2)
    yl = Y[:, rm[0] == rank]
    s = ScatterFunction.apply(yl, coo[[1]], rm[0], rm[1], 2, rank, world)
    exp = torch.zeros(4, 2).index_add_(0, coo[1], Y[0])
    torch.testing.assert_close(s[0], exp[2 * rank:2 * rank + 2])
    # comm-map exchange: rank r sends (p + 1) rows to peer p
    send = torch.full((1, sum(p + 1 for p in range(world)), 3), float(rank))
    recv = torch.empty(1, world * (rank + 1), 3)
    parts = torch_alltoallv_with_comm_map(send, recv, torch.arange(1, world + 1),
                                          torch.full((world,), rank + 1), rank, world)
    for p, t in enumerate(parts):
        assert torch.all(t == p)
    sd = {p: torch.full((p + 2, 3), float(rank)) for p in range(world) if p != rank}
    rd = {p: torch.empty(rank + 2, 3) for p in range(world) if p != rank}
    _nccl_alltoallv_with_dict(sd, rd, rank, world)
    for p, t in rd.items():
        assert torch.all(t == p)


def test_legacy_g1_functions(ranks):
    ranks(_legacy_fns, 2)
