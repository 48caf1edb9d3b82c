"""RGAT (the reference's OGB-LSC model, experiments/OGB-LSC/RGAT.py:271-382) on the lean fp32
path: ``CommAwareRGAT.forward(xs, HeteroGraph)`` — transform-first MFMA linears with the
skip and residual transforms folded into one weight, destination scores from the GEMM
(``V_r = a_dst W_r``), the fused relation attention of ops/gat.py added in place, halo rows
as a second source.

* W=1: forward and every parameter gradient against a plain-PyTorch RGAT written here
  from the model's own modules (per-edge scores, stable softmax, index_add);
* the relation attention op alone: fp64 gradcheck of its adjoint;
* W = 2 / 3 / 8 gloo ranks (layer 0 transforms the kept halo feature rows, layer 1
  exchanges transformed halo rows and returns their gradient) follow the W=1 losses;
* GPU: the three HIP kernels against the fp64 CPU run, and bitwise run to run.
"""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

from dgraph_amd.data.mag import (EDGE_TYPES, HETERO_SHAPES, build_hetero_partition,
                                 build_relation_csrs, hetero_node_data)
from dgraph_amd.models.rgat import CommAwareRGAT
from dgraph_amd.models.rgcn import HeteroGraph, layer_plan

SHAPE = HETERO_SHAPES["mag240m"].scaled(2e-5)


def _attention(h_dst, h_src, conv, csr):
    """Plain per-edge GAT of one relation (heads as channel blocks), fp64-safe."""
    H, C = conv.heads, conv.out_channels
    D = C // H
    hi, hj = conv.conv1(h_dst), conv.conv1(h_src)
    W = conv.project_message.weight
    rows, cols = csr.row_ids(), csr.col.long()
    e = torch.stack([(hi[rows, k * D:(k + 1) * D] * W[k, k * D:(k + 1) * D]).sum(-1) +
                     (hj[cols, k * D:(k + 1) * D] * W[k, C + k * D:C + (k + 1) * D]).sum(-1)
                     for k in range(H)], 1) + conv.project_message.bias
    e = F.leaky_relu(e, 0.2)
    mx = torch.full((csr.num_rows, H), -float("inf"), dtype=e.dtype).index_reduce(
        0, rows, e.detach(), "amax")
    p = torch.exp(e - mx[rows])
    den = torch.zeros(csr.num_rows, H, dtype=e.dtype).index_add(0, rows, p)
    a = p / den[rows]
    msg = (hj[cols].view(-1, H, D) * a.unsqueeze(-1)).reshape(-1, C)
    return torch.zeros(csr.num_rows, C, dtype=msg.dtype).index_add(0, rows, msg)


def _dense_reference(m, xs, csrs):
    need, rels = layer_plan(EDGE_TYPES, m.num_layers, 0)
    h = dict(xs)
    for l in range(m.num_layers):
        tmp = {t: m.skip_layers[l](h[t]) for t in need[l]}
        for r in rels[l]:
            s, d = EDGE_TYPES[r]
            conv = m.layers[l][r]
            tmp[d] = tmp[d] + _attention(h[d], h[s], conv, csrs[r]) + conv.res_net(h[d]) + \
                conv.bias
        h = {t: torch.relu(m.bn_layers[l](v)) for t, v in tmp.items()}
    return m.mlp(h[0])


def _model(cin, hid, layers, heads):
    torch.manual_seed(0)
    m = CommAwareRGAT(cin, SHAPE.num_classes, hid, 5, layers, heads, dropout=0.0)
    with torch.no_grad():  # non-trivial attention: random biases and score vectors
        for convs in m.layers:
            for c in convs:
                c.project_message.weight.normal_(0, 0.5)
                c.bias.normal_(0, 0.1)
    return m


@pytest.mark.parametrize("layers,heads", [(2, 1), (2, 4), (3, 2)])
def test_rgat_lean_matches_dense_reference(layers, heads):
    part = build_hetero_partition(SHAPE, 0, 1, "cpu", global_frac=0.2, window=64)
    g = HeteroGraph.from_partition(part, EDGE_TYPES)
    csrs, _ = build_relation_csrs(SHAPE, 0, 1, "cpu", global_frac=0.2, window=64)
    feats, y, tr = hetero_node_data(SHAPE, 0, part["offsets"], "cpu", dtype=torch.float32)
    feats = {t: v[:, :32].contiguous() for t, v in feats.items()}
    m = _model(32, 16, layers, heads)
    out = m(feats, g)
    F.cross_entropy(out[tr], y[tr]).backward()
    grads = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    ref = _dense_reference(m, feats, csrs)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-4)
    F.cross_entropy(ref[tr], y[tr]).backward()
    ref_grads = {n: p.grad for n, p in m.named_parameters() if p.grad is not None}
    assert grads.keys() == ref_grads.keys()
    for n, a in grads.items():
        torch.testing.assert_close(a, ref_grads[n], atol=2e-5, rtol=2e-4, msg=n)


def test_gat_relation_op_gradcheck():
    from dgraph_amd.ops.gat import GatPattern, gat_relation_into
    from dgraph_amd.ops.csr import CSR

    torch.manual_seed(1)
    R, N, C, H = 7, 9, 8, 2
    rows = torch.randint(0, R, (30,))
    cols = torch.randint(0, N, (30,))
    csr = CSR.from_coo(rows, cols, R, N)
    pat = GatPattern(csr.rowptr, csr.col, N, 0)
    z = torch.randn(N, C, dtype=torch.float64, requires_grad=True)
    sd = torch.randn(R, H, dtype=torch.float64, requires_grad=True)
    a = torch.randn(H, C // H, dtype=torch.float64, requires_grad=True)
    base = torch.randn(R, C, dtype=torch.float64, requires_grad=True)

    def f(z, sd, a, base):
        return gat_relation_into(z, sd, a, base * 1.0, pat)

    assert torch.autograd.gradcheck(f, (z, sd, a, base), eps=1e-6, atol=1e-6)


def _train(rank, world, steps, out, heads, static_halo=None, dev="cpu", width=24, hid=16):
    import torch.distributed as dist

    from dgraph_amd.parallel.grad_sync import GradSync

    if dev != "cpu":
        from conftest import rank_device

        dev = rank_device()
    # graph and data generated on the CPU (device RNG streams differ), then moved
    part = build_hetero_partition(SHAPE, rank, world, "cpu", global_frac=0.3, window=64)
    part = {k: v for k, v in part.items()}
    part["sources"] = {s: {k: (v.to(dev) if hasattr(v, "to") else v) for k, v in d.items()}
                       for s, d in part["sources"].items()}
    g = HeteroGraph.from_partition(part, EDGE_TYPES, rank=rank)
    feats, y, tr = hetero_node_data(SHAPE, rank, part["offsets"], "cpu", dtype=torch.float32)
    feats = {t: v[:, :width].contiguous().to(dev) for t, v in feats.items()}
    y, tr = y.to(dev), tr.to(dev)
    idx = torch.nonzero(tr).squeeze(1)
    n = torch.tensor([idx.numel()], device=dev if dist.is_initialized() and
                     dist.get_backend() == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(n)
    m = _model(width, hid, 2, heads).to(dev)
    m.static_halo = static_halo
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    sync = GradSync(m.parameters())
    losses = []
    for _ in range(steps):
        logits = m(feats, g)
        loss = F.cross_entropy(logits[idx], y[idx], reduction="sum") / n.item()
        loss.backward()
        sync.all_reduce()
        opt.step()
        opt.zero_grad()
        lt = loss.detach().clone().to(n.device)
        if world > 1:
            dist.all_reduce(lt)
        losses.append(float(lt))
    if rank == 0:
        torch.save(torch.tensor(losses), out)
    if dev != "cpu":
        from dgraph_amd.comm.alltoallv import close_shmem_heaps

        torch.cuda.synchronize()
        close_shmem_heaps()


@pytest.mark.parametrize("world,heads,static_halo", [(2, 4, None), (3, 1, None), (8, 2, None),
                                                    (2, 4, False), (3, 2, False)])
def test_rgat_lean_distributed_matches_single_rank(ranks, tmp_path, world, heads, static_halo):
    """(``static_halo=False``: layer 0 exchanges each relation's transformed halo rows per
    step and returns their gradient, instead of transforming kept feature halo rows.)"""
    _train(0, 1, 3, tmp_path / "w1.pt", heads)
    ranks(_train, world, 3, str(tmp_path / "wn.pt"), heads, static_halo)
    a = torch.load(tmp_path / "w1.pt", weights_only=True)
    b = torch.load(tmp_path / "wn.pt", weights_only=True)
    torch.testing.assert_close(a, b, atol=2e-5, rtol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("static_halo", [None, False])
def test_rgat_lean_two_processes_one_gpu(monkeypatch, tmp_path, static_halo):
    """W=2 on the GPU kernels (two processes sharing the GPU, halo exchanges on the IPC
    heap): layer 0 with the kept feature halo or with exchanged transformed halo rows —
    rebuilt in backward (remake: z recomputed by the same GEMM, its halo rows received
    again) — follows the W=1 losses of the same GPU model."""
    from conftest import run_ranks

    monkeypatch.setenv("DGRAPH_A2A_IMPL", "shmem")
    monkeypatch.setenv("DGRAPH_SYMHEAP_BYTES", str(256 << 20))
    _train(0, 1, 3, tmp_path / "w1.pt", 4, None, "cuda", 64, 64)
    run_ranks(_train, 2, 3, str(tmp_path / "w2.pt"), 4, static_halo, "cuda", 64, 64,
              timeout=240)
    a = torch.load(tmp_path / "w1.pt", weights_only=True)
    b = torch.load(tmp_path / "w2.pt", weights_only=True)
    torch.testing.assert_close(a, b, atol=2e-5, rtol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("width,heads", [(64, 1), (128, 4), (128, 2), (256, 4), (256, 8)])
def test_rgat_lean_gpu_matches_fp64_cpu(width, heads):
    """The fused attention kernels (csrc/kernels/gat_f32.hip) and the exact-f32 MFMA linears
    against the same model run on the CPU in fp64 attention; then bitwise run to run."""
    shape = HETERO_SHAPES["mag240m"].scaled(1e-4)
    part_cpu = build_hetero_partition(shape, 0, 1, "cpu", global_frac=0.2, window=256)
    feats_cpu, y_cpu, tr_cpu = hetero_node_data(shape, 0, part_cpu["offsets"], "cpu",
                                                dtype=torch.float32)
    res = {}
    for dev in ("cpu", "cuda", "cuda"):
        part = {"offsets": part_cpu["offsets"], "sources": {
            s: {k: (v.to(dev) if hasattr(v, "to") else v) for k, v in d.items()}
            for s, d in part_cpu["sources"].items()}}
        g = HeteroGraph.from_partition(part, EDGE_TYPES)
        feats = {t: v[:, :width].to(dev).contiguous() for t, v in feats_cpu.items()}
        y, tr = y_cpu.to(dev), tr_cpu.to(dev)
        m = _model(width, width, 2, heads).to(dev)
        m.remake_layer0 = True  # (the W>1 default: layer-0 z rebuilt in backward)
        out = m(feats, g)
        F.cross_entropy(out[tr], y[tr]).backward()
        got = (out.detach().cpu(), {n: p.grad.cpu() for n, p in m.named_parameters()
                                    if p.grad is not None})
        if dev in res:
            # bitwise run to run (fixed summation orders, no atomics)
            assert torch.equal(got[0], res[dev][0])
            for n, t in got[1].items():
                assert torch.equal(t, res[dev][1][n]), n
        res[dev] = got
    torch.testing.assert_close(res["cuda"][0], res["cpu"][0], atol=1e-3, rtol=1e-3)
    assert res["cuda"][1].keys() == res["cpu"][1].keys()
    for n, b in res["cpu"][1].items():
        a = res["cuda"][1][n]
        rel = float((a - b).norm() / b.norm().clamp_min(1e-4))
        assert rel < 1e-3, (n, rel)


@pytest.mark.gpu
@pytest.mark.parametrize("C,heads", [(256, 4), (128, 2), (256, 2)])
def test_gat_head_passes_match_whole_rows(monkeypatch, C, heads):
    """One kernel pass per head over its column slice (ops/gat.py HEAD_PASSES) against one
    pass over whole rows: same forward and gradients to fp32 rounding (the per-head softmax
    sums are grouped differently), two sources (a halo part) included."""
    import dgraph_amd.ops.gat as G
    from dgraph_amd.ops.csr import CSR

    torch.manual_seed(3)
    R, N, H, E = 3000, 2500, 700, 60000
    rows = torch.randint(0, R, (E,))
    cols = torch.randint(0, N + H, (E,))
    csr = CSR.from_coo(rows, cols, R, N + H)
    dev = torch.device("cuda")
    pat = G.GatPattern(csr.rowptr.to(dev), csr.col.to(dev), N, H)
    z0 = torch.randn(N, C, device=dev)
    zh = torch.randn(H, C, device=dev)
    sd0 = torch.randn(R, heads, device=dev)
    a0 = torch.randn(heads, C // heads, device=dev) * 0.3
    base = torch.randn(R, C, device=dev)
    w = torch.randn(R, C, device=dev)
    res = {}
    for hp in (True, False):
        monkeypatch.setattr(G, "HEAD_PASSES", hp)
        z = z0.clone().requires_grad_()
        sd = sd0.clone().requires_grad_()
        a = a0.clone().requires_grad_()
        out = G.gat_relation_into(z, sd, a, base.clone(), pat, zh_static=zh)
        (out * w).sum().backward()
        res[hp] = (out.detach(), z.grad, sd.grad, a.grad)
    for x, y in zip(res[True], res[False]):
        torch.testing.assert_close(x, y, rtol=2e-5, atol=2e-5)
