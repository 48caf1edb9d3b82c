"""``act_linears`` (BN + ReLU + dropout recomputed in backward, several linears of one
activation) against the composition of the modules it replaces, and the in-place source
aggregation against aggregate-then-add — forward and every gradient, CPU fp32/fp64."""
from __future__ import annotations

import pytest
import torch

from dgraph_amd.models.norm import DistributedBatchNorm1D
from dgraph_amd.ops.act_linear import act_linears


@pytest.mark.parametrize("dropout", [0.0, 0.3])
@pytest.mark.parametrize("with_bn", [True, False])
def test_act_linears_matches_composition(with_bn, dropout):
    torch.manual_seed(0)
    M, K = 300, 24
    x = torch.randn(M, K, dtype=torch.float64, requires_grad=True)
    Ws = [torch.randn(n, K, dtype=torch.float64, requires_grad=True) for n in (16, 40)]
    b = torch.randn(16, dtype=torch.float64, requires_grad=True)
    bn = DistributedBatchNorm1D(K).double() if with_bn else None
    if bn is not None:
        with torch.no_grad():
            bn.gamma.uniform_(0.5, 1.5)
            bn.beta.uniform_(-0.5, 0.5)
    d = dropout if with_bn else 0.0
    g = [torch.randn(M, 16, dtype=torch.float64), torch.randn(M, 40, dtype=torch.float64)]

    def run(fused):
        for t in [x, b, *Ws] + ([bn.gamma, bn.beta] if bn is not None else []):
            t.grad = None
        torch.manual_seed(7)  # the same dropout seed for both
        if fused:
            outs = act_linears(x, Ws, b, bn=bn, relu=with_bn, dropout=d)
        else:
            y = bn(x, relu=True, dropout=d) if bn is not None else x
            outs = [torch.nn.functional.linear(y, Ws[0], b), y @ Ws[1].t()]
        sum((o * gg).sum() for o, gg in zip(outs, g)).backward()
        grads = [t.grad.clone() for t in [x, b, *Ws]]
        if bn is not None:
            grads += [bn.gamma.grad.clone(), bn.beta.grad.clone()]
        return [o.detach() for o in outs], grads, (None if bn is None else
                                                    bn.running_var.clone())

    o1, g1, rv1 = run(True)
    o2, g2, rv2 = run(False)
    for a, c in zip(o1, o2):
        torch.testing.assert_close(a, c)
    for a, c in zip(g1, g2):
        torch.testing.assert_close(a, c)


def test_act_linears_eval_mode_uses_running_stats():
    torch.manual_seed(0)
    bn = DistributedBatchNorm1D(8)
    bn.eval()
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
    x = torch.randn(20, 8)
    W = torch.randn(4, 8)
    out = act_linears(x, [W], bn=bn, relu=True)[0]
    torch.testing.assert_close(out, bn(x, relu=True) @ W.t())


def test_source_aggregate_into_matches_aggregate_plus_add():
    from dgraph_amd.data.mag import EDGE_TYPES, HETERO_SHAPES, build_hetero_partition
    from dgraph_amd.models.rgcn import HeteroGraph
    from dgraph_amd.parallel.hetero_graph import source_aggregate, source_aggregate_into

    shape = HETERO_SHAPES["mag240m"].scaled(2e-5)
    part = build_hetero_partition(shape, 0, 1, "cpu", global_frac=0.2, window=64)
    g = HeteroGraph.from_partition(part, EDGE_TYPES)
    s = 0  # papers: cites (-> papers) and written-by (-> authors)
    sg = g.sources[s]
    rs = sorted(sg.ranges)
    C = 8
    torch.manual_seed(0)
    z = torch.randn(sg.Ls, C * len(rs), dtype=torch.float64, requires_grad=True)
    spec = [(r, i * C, (i + 1) * C) for i, r in enumerate(rs)]
    n = {r: sg.ranges[r][1] - sg.ranges[r][0] for r in rs}
    base = {r: torch.randn(n[r], C, dtype=torch.float64, requires_grad=True) for r in rs}
    gs = {r: torch.randn(n[r], C, dtype=torch.float64) for r in rs}

    outs = source_aggregate(z, sg, spec)
    ref = [base[r] + o for r, o in zip(rs, outs)]
    sum((o * gs[r]).sum() for r, o in zip(rs, ref)).backward()
    gz_ref = z.grad.clone()
    gb_ref = {r: base[r].grad.clone() for r in rs}
    z.grad = None
    for r in rs:
        base[r].grad = None

    tg = [base[r].clone() for r in rs]  # in place: clones of the leaves
    got = source_aggregate_into(z, sg, spec, tg)
    for a, c in zip(got, ref):
        torch.testing.assert_close(a, c.detach())
    sum((o * gs[r]).sum() for r, o in zip(rs, got)).backward()
    torch.testing.assert_close(z.grad, gz_ref)
    for r in rs:
        torch.testing.assert_close(base[r].grad, gb_ref[r])
