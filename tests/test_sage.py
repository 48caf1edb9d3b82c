"""GraphSAGE model numerics (CPU reference path) vs a dense-adjacency reference, and
distributed training equivalence across world sizes on gloo."""
import pytest
import torch

from dgraph_amd.data.synthetic import SHAPES, build_partition, node_data
from dgraph_amd.models.sage import GraphSAGE, SAGEConv
from dgraph_amd.parallel.dist_graph import DistGraph

SHAPE = SHAPES["ogbn-arxiv"].scaled(0.01)


def _graph():
    p = build_partition(SHAPE, 0, 1, "cpu")
    csr = p["csr"]
    A = torch.zeros(p["L"], p["L"])
    A.index_put_((csr.row_ids(), csr.col.long()), torch.ones(csr.nnz), accumulate=True)
    A = A / A.sum(1, keepdim=True).clamp(min=1)
    return p, DistGraph(csr, p["L"], 0, symmetric=True), A


def _dense_forward(m, x, A):
    h = x
    for l in m.layers:
        h = h @ l.w_self + (A @ h) @ l.w_neigh + l.bias
        if l.relu:
            h = h.relu()
    return h


@pytest.mark.parametrize("hidden,classes", [(64, 40), (60, 37), (128, 172)])
@pytest.mark.parametrize("subset", [True, False])
def test_stack_matches_dense(hidden, classes, subset):
    p, g, A = _graph()
    x, _, tr = node_data(SHAPE, 0, p["offsets"], "cpu", dtype=torch.float32)
    torch.manual_seed(0)
    m = GraphSAGE(SHAPE.num_features, hidden, classes, 3)
    rows = torch.nonzero(tr).squeeze(1) if subset else None
    out = m(x, g, out_rows=rows)
    out.square().mean().backward()
    grads = [q.grad.clone() for q in m.parameters()]
    m.zero_grad()
    ref = _dense_forward(m, x, A)
    ref = ref[rows] if subset else ref
    ref.square().mean().backward()
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-4)
    for a, q in zip(grads, m.parameters()):
        torch.testing.assert_close(a, q.grad, atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("order", ["aggregate_first", "project_first"])
@pytest.mark.parametrize("save", [True, False])
def test_sageconv_backward_variants(order, save):
    p, g, A = _graph()
    x = torch.randn(p["L"], 32, requires_grad=True)
    c = SAGEConv(32, 48, order=order, save_agg=save)
    c(x, g).square().sum().backward()
    gx = x.grad.clone()
    gw = [q.grad.clone() for q in c.parameters()]
    x.grad = None
    c.zero_grad()
    (x @ c.w_self + (A @ x) @ c.w_neigh + c.bias).relu().square().sum().backward()
    torch.testing.assert_close(gx, x.grad, atol=1e-4, rtol=1e-4)
    for a, q in zip(gw, c.parameters()):
        torch.testing.assert_close(a, q.grad, atol=1e-3, rtol=1e-4)


def test_workspace_guard():
    p, g, _ = _graph()
    x, _, _ = node_data(SHAPE, 0, p["offsets"], "cpu", dtype=torch.float32)
    m = GraphSAGE(SHAPE.num_features, 32, 8, 2)
    rows = torch.arange(10)
    o1 = m(x, g, out_rows=rows)
    m(x, g, out_rows=rows)  # second forward reuses the workspace
    with pytest.raises(RuntimeError, match="workspace"):
        o1.sum().backward()


def _train_losses(rank, world, steps, out, hidden=32):
    import torch.distributed as dist

    from dgraph_amd.parallel.grad_sync import GradSync

    p = build_partition(SHAPE, rank, world, "cpu")
    g = DistGraph(p["csr"], p["L"], p["H"], p["send_local_idx"], p["send_splits"],
                  p["recv_splits"], symmetric=(world == 1))
    x, y, tr = node_data(SHAPE, rank, p["offsets"], "cpu", dtype=torch.float32)
    idx = torch.nonzero(tr).squeeze(1)
    n = torch.tensor([idx.numel()])
    if world > 1:
        dist.all_reduce(n)
    torch.manual_seed(0)
    m = GraphSAGE(SHAPE.num_features, hidden, SHAPE.num_classes, 3)
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    sync = GradSync(m.parameters())
    losses = []
    for _ in range(steps):
        logits = m(x, g, out_rows=idx)
        loss = torch.nn.functional.cross_entropy(logits, y[idx], reduction="sum") / n.item()
        loss.backward()
        sync.all_reduce()
        opt.step()
        opt.zero_grad()
        lt = loss.detach().clone()
        if world > 1:
            dist.all_reduce(lt)
        losses.append(float(lt))
    if rank == 0:
        torch.save(torch.tensor(losses), out)


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("hidden", [32, 64])
def test_distributed_training_matches_single_rank(ranks, tmp_path, world, hidden):
    """Halo-overlapped DistGraph training on W ranks follows the same loss curve as W=1.
    hidden=64 > 40 classes makes the output layer project-first: its backward takes the
    row-restricted path with the contributing-rows reverse exchange."""
    _train_losses(0, 1, 4, tmp_path / "w1.pt", hidden)
    ranks(_train_losses, world, 4, str(tmp_path / "wn.pt"), hidden)
    a = torch.load(tmp_path / "w1.pt", weights_only=True)
    b = torch.load(tmp_path / "wn.pt", weights_only=True)
    torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("keep_agg0", [True, False])
def test_layer0_aggregate_kept_or_recomputed(monkeypatch, keep_agg0):
    from dgraph_amd.models.sage import SageWorkspace

    if not keep_agg0:  # no room for the slot: backward recomputes A x0
        monkeypatch.setattr(SageWorkspace, "AGG0_HEADROOM", 1 << 62)
    p, g, A = _graph()
    x, _, tr = node_data(SHAPE, 0, p["offsets"], "cpu", dtype=torch.float32)
    torch.manual_seed(0)
    m = GraphSAGE(SHAPE.num_features, 256, 40, 3)  # layer 0 aggregates first
    rows = torch.nonzero(tr).squeeze(1)
    m(x, g, out_rows=rows).square().mean().backward()
    assert m._workspace.has("agg0") == keep_agg0
    grads = [q.grad.clone() for q in m.parameters()]
    m.zero_grad()
    _dense_forward(m, x, A)[rows].square().mean().backward()
    for a, q in zip(grads, m.parameters()):
        torch.testing.assert_close(a, q.grad, atol=1e-6, rtol=1e-4)


def _static_halo(rank, world):
    from dgraph_amd.comm.alltoallv import CommStats

    p = build_partition(SHAPE, rank, world, "cpu")
    g = DistGraph(p["csr"], p["L"], p["H"], p["send_local_idx"], p["send_splits"],
                  p["recv_splits"])
    x, _, _ = node_data(SHAPE, rank, p["offsets"], "cpu", dtype=torch.float32)
    ref = g.aggregate(x)
    c0 = CommStats.calls
    a = g.aggregate(x, static=True)
    b = g.aggregate(x, static=True)
    assert CommStats.calls == c0 + 1  # exchanged once, then reused
    torch.testing.assert_close(a, ref)
    torch.testing.assert_close(b, ref)
    x.mul_(2.0)  # in-place update: version bump -> re-exchange
    torch.testing.assert_close(g.aggregate(x, static=True), 2.0 * ref)
    assert CommStats.calls == c0 + 2
    y = x.clone()  # a different tensor with equal contents
    torch.testing.assert_close(g.aggregate(y, static=True), 2.0 * ref)
    assert CommStats.calls == c0 + 3


def test_static_feature_halo_cached(ranks):
    ranks(_static_halo, 2)


@pytest.mark.parametrize("classes", [40, 172])
def test_eval_rows_and_restricted_last_layer(classes):
    """The full-graph step returns validation/test logits from the same forward
    (``eval_rows``), and the train-rows-only variant (``restrict_last``) produces the same
    loss-row logits and gradients as the full output layer."""
    p, g, A = _graph()
    x, _, tr = node_data(SHAPE, 0, p["offsets"], "cpu", dtype=torch.float32)
    rows = torch.nonzero(tr).squeeze(1)
    ev_rows = torch.nonzero(~tr).squeeze(1)[::3]
    res = {}
    for restrict in (False, True):
        torch.manual_seed(0)
        m = GraphSAGE(SHAPE.num_features, 64, classes, 3)
        if restrict:
            out = m(x, g, out_rows=rows, restrict_last=True)
            ev = None
        else:
            out, ev = m(x, g, out_rows=rows, eval_rows=ev_rows)
            assert not ev.requires_grad
        out.square().mean().backward()
        res[restrict] = (out.detach(), ev, [q.grad.clone() for q in m.parameters()], m)
    full = _dense_forward(res[False][3], x, A).detach()
    torch.testing.assert_close(res[False][1], full[ev_rows], atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(res[True][0], res[False][0], atol=1e-5, rtol=1e-4)
    for a, b in zip(res[True][2], res[False][2]):
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-4)
    with pytest.raises(ValueError):
        res[True][3](x, g, out_rows=rows, eval_rows=ev_rows, restrict_last=True)


@pytest.mark.parametrize("hidden,classes", [(64, 40), (96, 47)])
def test_grad_support_matches_dense(hidden, classes):
    """With the gradient support prepared (DistGraph.prepare_grad_support), the layer
    below the loss-row-sparse output layer aggregates transposed only from the loss rows
    and their neighbours: same gradients as dense autograd, fewer edges aggregated."""
    p, g, A = _graph()
    x, _, tr = node_data(SHAPE, 0, p["offsets"], "cpu", dtype=torch.float32)
    rows = torch.nonzero(tr).squeeze(1)[:8]  # a few loss rows: a small support
    sup = g.prepare_grad_support(rows)
    assert sup is not None and sup[1].nnz < g.nnz
    torch.manual_seed(0)
    m = GraphSAGE(SHAPE.num_features, hidden, classes, 3)
    e0 = g.edges_aggregated
    out = m(x, g, out_rows=rows)
    out.square().mean().backward()
    e_sup = g.edges_aggregated - e0
    grads = [q.grad.clone() for q in m.parameters()]
    m.zero_grad()
    ref = _dense_forward(m, x, A)[rows]
    ref.square().mean().backward()
    for a, q in zip(grads, m.parameters()):
        torch.testing.assert_close(a, q.grad, atol=1e-6, rtol=1e-4)
    g.GRAD_SUPPORT = False
    g._support_cache.clear()
    e0 = g.edges_aggregated
    m(x, g, out_rows=rows).square().mean().backward()
    assert e_sup < g.edges_aggregated - e0
