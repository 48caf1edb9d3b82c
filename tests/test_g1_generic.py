"""Index-based API (G1) at any world size, against a replicated ground truth.

The literal 2-rank graphs of the reference's backend tests live in test_g1_backends.py;
these bodies generate a random graph whose size grows with W (so W=8 exercises 8-way
splits, empty peers and uneven degree) and check every engine's gather / scatter (and the
gather backward) against the same computation on the whole replicated graph
(the reference's ground-truth style, tests/test_NCCLCommPlan.py:85-124)."""
import pytest
import torch

N_PER, E_PER, F = 3, 7, 5


def _graph(world):
    g = torch.Generator().manual_seed(11 + world)
    N, E = N_PER * world, E_PER * world
    coo = torch.randint(0, N, (2, E), generator=g)
    X = torch.randn(1, N, F, generator=g)
    Xe = torch.randn(1, E, F, generator=g)
    return N, E, coo, X, Xe


def _nccl_body(rank, world):
    from dgraph_amd import Communicator

    comm = Communicator.init_process_group("nccl")
    try:
        N, E, coo, X, Xe = _graph(world)
        owner = coo // N_PER               # vertex owner of each endpoint
        edge_place = owner[0]              # an edge lives with its coo[0] endpoint
        xl = comm.get_local_rank_slice(X)
        assert torch.equal(xl, X[:, N_PER * rank:N_PER * (rank + 1)])
        mine = edge_place == rank
        for i in range(2):
            m = torch.stack([edge_place, owner[i]])
            xg = xl.clone().requires_grad_(True)
            got = comm.gather(xg, coo[[i]], m)
            torch.testing.assert_close(got[0], X[0, coo[i]][mine])
            # backward = scatter-sum of the edge gradients onto the owned vertices
            w = torch.arange(1.0, got.shape[1] + 1).reshape(1, -1, 1).expand_as(got)
            (got * w).sum().backward()
            full = torch.zeros(N, F).index_add_(
                0, coo[i][mine], w[0] if got.shape[1] else torch.zeros(0, F))
            if world > 1:
                import torch.distributed as dist

                dist.all_reduce(full)
            torch.testing.assert_close(xg.grad[0], full[N_PER * rank:N_PER * (rank + 1)])
            # scatter: the edges placed here are summed into their (remote) owners
            xe = comm.get_local_tensor(Xe, edge_place, dim=1)
            got_s = comm.scatter(xe, coo[[i]], m, N_PER)
            exp = torch.zeros(N, F).index_add_(0, coo[i], Xe[0])
            torch.testing.assert_close(got_s[0], exp[N_PER * rank:N_PER * (rank + 1)])
    finally:
        comm.destroy()


def _edge_block_body(rank, world, backend):
    """mpi / rocshmem engines: edges are block-partitioned (E_PER per rank)."""
    from dgraph_amd import Communicator

    comm = Communicator.init_process_group(backend, SKIP_NCCL_ASSERT=True)
    try:
        N, E, coo, X, Xe = _graph(world)
        owner = coo // N_PER
        xl = comm.get_local_rank_slice(X, dim=1)
        lo, hi = E_PER * rank, E_PER * (rank + 1)
        for i in range(2):
            li = comm.get_local_rank_slice(coo[[i]], dim=1)
            lm = comm.get_local_rank_slice(owner[[i]], dim=1)
            assert torch.equal(li[0], coo[i, lo:hi])
            got = comm.gather(xl, li, lm)
            torch.testing.assert_close(got, X[:, coo[i]][:, lo:hi])
            xs = comm.get_local_rank_slice(Xe, dim=1)
            # the reference's engines disagree on the argument order (MPIBackendEngine
            # scatter(x, idx, n, map) vs NVSHMEMBackendEngine scatter(x, idx, map, n))
            got_s = (comm.scatter(xs, li, N_PER, lm) if backend == "mpi"
                     else comm.scatter(xs, li, lm, N_PER))
            exp = torch.zeros(N, F).index_add_(0, coo[i], Xe[0])
            torch.testing.assert_close(got_s[0], exp[N_PER * rank:N_PER * (rank + 1)])
    finally:
        comm.destroy()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_nccl_g1_any_world(ranks, world):
    ranks(_nccl_body, world)


@pytest.mark.parametrize("backend", ["mpi", "rocshmem"])
@pytest.mark.parametrize("world", [2, 8])
def test_edge_block_engines_any_world(ranks, world, backend):
    ranks(_edge_block_body, world, backend)
