"""HaloExchange / DGraphMessagePassing (G3) forward + backward on gloo at W=2..4 and on
every engine that implements ``put`` (the reference only had it on NCCL, D3)."""
import pytest
import torch

from dgraph_amd.plan.pattern import build_communication_pattern


def _graph(seed=0, V=48, E=300):
    g = torch.Generator().manual_seed(seed)
    e = torch.randint(0, V, (E, 2), generator=g)
    e = torch.cat([e, e.flip(1)])
    return V, e


class SumConv(torch.nn.Module):
    """out[i] = sum_{(i,j)} W x_j  (central i local, neighbour j local or halo)."""

    def __init__(self, F):
        super().__init__()
        self.lin = torch.nn.Linear(F, F, bias=False)
        torch.nn.init.eye_(self.lin.weight)

    def forward(self, x, edges, ef=None):
        n_local = int(edges[:, 0].max()) + 1 if edges.numel() else 0
        msg = self.lin(x[edges[:, 1]])
        out = torch.zeros(self._L, x.shape[1], dtype=x.dtype)
        return out.index_add(0, edges[:, 0], msg)


def _halo(rank, world, backend):
    from dgraph_amd import Communicator
    from dgraph_amd.parallel.halo import DGraphMessagePassing, HaloExchange

    comm = Communicator.init_process_group(backend)
    try:
        V, E = _graph()
        part = torch.randint(0, world, (V,), generator=torch.Generator().manual_seed(1))
        cp = build_communication_pattern(E, part, rank, world)
        X = torch.randn(V, 6, generator=torch.Generator().manual_seed(2))
        lv = cp.local_vertices
        xl = X[lv].clone().requires_grad_(True)
        halo = HaloExchange(comm)(xl, cp)
        torch.testing.assert_close(halo, X[cp.halo_vertices])
        # backward: d/dX of sum_e w_e * halo -> each vertex receives grads from every
        # rank it was sent to
        w = torch.randn(halo.shape, generator=torch.Generator().manual_seed(3 + rank))
        (halo * w).sum().backward()
        # ground truth assembled from all ranks' (halo_ids, w)
        gX = torch.zeros(V, 6)
        for r in range(world):
            cp_r = _pattern_offline(E, part, r, world)
            w_r = torch.randn((cp_r.numel(), 6), generator=torch.Generator().manual_seed(3 + r))
            gX.index_add_(0, cp_r, w_r)
        torch.testing.assert_close(xl.grad, gX[lv], atol=1e-5, rtol=1e-5)
        # full message-passing layer
        conv = SumConv(6)
        conv._L = cp.num_local_vertices
        mp = DGraphMessagePassing(HaloExchange(comm), conv)
        out = mp(X[lv], cp)
        ref = torch.zeros(V, 6).index_add(0, E[:, 0], X[E[:, 1]])
        torch.testing.assert_close(out, ref[lv], atol=1e-5, rtol=1e-5)
    finally:
        comm.destroy()


def _pattern_offline(E, part, r, world):
    """Halo ids of rank r in receive order = sorted (owner, gid) of remote neighbours."""
    mine = E[part[E[:, 0]] == r]
    nb = mine[:, 1]
    rem = part[nb] != r
    V = part.numel()
    key = torch.unique(part[nb[rem]] * V + nb[rem])
    return key % V


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_halo_exchange_nccl(ranks, world):
    ranks(_halo, world, "nccl")


@pytest.mark.parametrize("backend", ["mpi", "rocshmem"])
def test_halo_exchange_other_backends(ranks, backend):
    ranks(_halo, 2, backend)


def test_halo_exchange_single_rank():
    from dgraph_amd.parallel.halo import HaloExchange

    class Fake:
        def alloc_buffer(self, size, dtype, device):
            return torch.empty(size, dtype=dtype, device=device)

        def put(self, *a, **k):
            pass

    V, E = _graph()
    cp = build_communication_pattern(E, torch.zeros(V, dtype=torch.long), 0, 1)
    x = torch.randn(V, 3, requires_grad=True)
    h = HaloExchange(Fake())(x, cp)
    assert h.shape == (0, 3)


def _async_halo(rank, world):
    """AsyncHalo (issue, independent work, wait) equals the synchronous HaloExchange,
    forward and backward (the send rows' gradient arrives through the reverse exchange
    issued from the halo gradient)."""
    from dgraph_amd import Communicator
    from dgraph_amd.parallel.halo import AsyncHalo, HaloExchange

    comm = Communicator.init_process_group("nccl")
    try:
        V, E = _graph(seed=3)
        part = torch.randint(0, world, (V,), generator=torch.Generator().manual_seed(4))
        cp = build_communication_pattern(E, part, rank, world)
        L = cp.num_local_vertices
        g = torch.Generator().manual_seed(10 + rank)
        x0 = torch.randn(L, 5, generator=g, dtype=torch.float64)
        wh = torch.randn(cp.num_halo_vertices, 5, generator=g, dtype=torch.float64)
        res = []
        for mode in ("sync", "async"):
            x = x0.clone().requires_grad_()
            if mode == "sync":
                halo = HaloExchange(comm)(x, cp)
            else:
                h = AsyncHalo.start(comm, x, cp)
                local_work = (x * 2).sum()  # independent work while the exchange is pending
                halo = h.wait()
            loss = (halo * wh).sum() + (x ** 2).sum() + (local_work if mode == "async" else 0)
            loss.backward()
            grad = x.grad.clone() - (2.0 if mode == "async" else 0.0)
            res.append((halo.detach().clone(), grad))
        assert torch.equal(res[0][0], res[1][0])
        torch.testing.assert_close(res[1][1], res[0][1])
    finally:
        comm.destroy()


@pytest.mark.parametrize("world", [2, 3])
def test_async_halo_matches_sync(ranks, world):
    ranks(_async_halo, world)
