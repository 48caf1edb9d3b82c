"""Numerics of the native HIP kernels vs the fp32 PyTorch reference of the same op.

The reference's kernel tests (tests/test_local_kernels.py) used F=4 only, so only its
float4 kernel was ever exercised; here every vector width, odd F, bf16, int32/int64
indices, heads, scales, accumulate and empty inputs are covered.
"""
import pytest
import torch

from dgraph_amd.ops import kernels as K
from dgraph_amd.ops import reference as R
from dgraph_amd.ops.csr import CSR

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rand_csr(R_, C, avg_deg, idx_dtype, device, skew=False, seed=0):
    g = torch.Generator().manual_seed(seed)
    deg = torch.poisson(torch.full((R_,), float(avg_deg)), generator=g).long()
    if skew and R_ > 3:
        deg[0] = 5000
        deg[R_ // 2] = 0
    rowptr = torch.zeros(R_ + 1, dtype=torch.long)
    rowptr[1:] = torch.cumsum(deg, 0)
    col = torch.randint(0, C, (int(rowptr[-1]),), generator=g)
    return CSR(rowptr.to(device), col.to(idx_dtype).to(device), C)


def _tol(dtype):
    return dict(atol=2e-2, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("F", [1, 3, 4, 8, 16, 100, 128, 172, 256, 600])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
def test_spmm_matches_reference(F, dtype, idx):
    csr = _rand_csr(300, 257, 7, idx, DEV, skew=True, seed=F)
    g = torch.Generator().manual_seed(F)
    x = torch.randn(257, F, generator=g).to(dtype).to(DEV)
    rs = torch.rand(300, generator=g).to(DEV)
    cs = torch.rand(257, generator=g).to(DEV)
    out = K.spmm(csr.rowptr, csr.col, x, row_scale=rs, col_scale=cs)
    ref = R.spmm(csr.rowptr.cpu(), csr.col.cpu(), x.double().cpu(),
                 torch.empty(300, F, dtype=torch.float64), None, cs.cpu(), rs.cpu()).float()
    # row 0 sums 5000 terms: fp32 summation-order error reaches ~1e-4 absolute there
    tol = _tol(dtype) if dtype == torch.bfloat16 else dict(atol=5e-4, rtol=1e-4)
    torch.testing.assert_close(out.float().cpu(), ref, **tol)


@pytest.mark.parametrize("heads,F", [(1, 64), (4, 64), (8, 128), (2, 6)])
def test_spmm_edge_weights_heads_and_beta(heads, F):
    csr = _rand_csr(200, 150, 5, torch.int32, DEV, seed=heads)
    x = torch.randn(150, F, device=DEV)
    ew = torch.rand(csr.nnz, heads, device=DEV)
    base = torch.randn(200, F, device=DEV)
    out = base.clone()
    K.spmm(csr.rowptr, csr.col, x, out, edge_weight=ew, heads=heads, beta=0.5)
    ref = R.spmm(csr.rowptr.cpu(), csr.col.cpu(), x.cpu(), base.cpu().clone(), ew.cpu(),
                 None, None, heads, 0.5)
    torch.testing.assert_close(out.cpu(), ref, atol=1e-4, rtol=1e-4)


def test_spmm_strided_and_empty():
    csr = _rand_csr(50, 40, 0, torch.int32, DEV)  # all rows empty
    x = torch.randn(40, 32, device=DEV)
    out = K.spmm(csr.rowptr, csr.col, x)
    assert torch.count_nonzero(out) == 0
    csr = _rand_csr(50, 40, 4, torch.int64, DEV)
    big = torch.randn(40, 48, device=DEV)
    xs = big[:, 8:40]  # row stride 48, feature stride 1
    out = K.spmm(csr.rowptr, csr.col, xs)
    ref = R.spmm(csr.rowptr.cpu(), csr.col.cpu(), xs.cpu(), torch.empty(50, 32))
    torch.testing.assert_close(out.cpu(), ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("variant,xcd", [(1, 0), (2, 0), (2, 1), (2, 2), (2, 3)])
@pytest.mark.parametrize("F", [16, 40, 64, 128, 256])
def test_spmm_variants_agree_ragged_rows(variant, xcd, F):
    """Rows whose degrees are not multiples of the lane-group count and exceed one
    64-edge chunk (exercises every group finishing at a different slot)."""
    from dgraph_amd import _native

    g = torch.Generator().manual_seed(F)
    deg = torch.randint(0, 200, (700,), generator=g)
    rowptr = torch.zeros(701, dtype=torch.long)
    rowptr[1:] = torch.cumsum(deg, 0)
    col = torch.randint(0, 500, (int(rowptr[-1]),), generator=g, dtype=torch.int32)
    x = torch.randn(500, F, device=DEV)
    ref = R.spmm(rowptr, col, x.cpu(), torch.empty(700, F))
    ops = _native.ops()
    try:
        ops.set_spmm_config(variant, xcd)
        out = K.spmm(rowptr.to(DEV), col.to(DEV), x)
    finally:
        ops.set_spmm_config(-1, -1)
    torch.testing.assert_close(out.cpu(), ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("variant,xcd", [(2, 2), (2, 0), (4, 2), (4, 0)])
@pytest.mark.parametrize("F", [8, 40, 64, 128, 192, 256, 520])
@pytest.mark.parametrize("mode", ["row", "col", "ew_beta"])
def test_spmm_bf16_variants_ragged(variant, xcd, F, mode):
    """bf16 kernels (v3 packed math, v4 row groups) on ragged degrees 0..199, every
    weighting mode, against the fp32 reference."""
    from dgraph_amd import _native

    g = torch.Generator().manual_seed(F + variant)
    deg = torch.randint(0, 200, (301,), generator=g)
    deg[::17] = 0
    rowptr = torch.zeros(302, dtype=torch.long)
    rowptr[1:] = torch.cumsum(deg, 0)
    col = torch.randint(0, 500, (int(rowptr[-1]),), generator=g, dtype=torch.int32)
    x = torch.randn(500, F, generator=g).to(torch.bfloat16)
    kw, rkw = {}, {}
    out0 = None
    if mode == "row":
        rs = torch.rand(301, generator=g)
        kw, rkw = {"row_scale": rs.to(DEV)}, {"row_scale": rs}
    elif mode == "col":
        cs = torch.rand(500, generator=g)
        kw, rkw = {"col_scale": cs.to(DEV)}, {"col_scale": cs}
    else:
        ew = torch.rand(col.numel(), generator=g)
        out0 = torch.randn(301, F, generator=g).to(torch.bfloat16)
        kw, rkw = {"edge_weight": ew.to(DEV), "beta": 0.5}, {"edge_weight": ew, "beta": 0.5}
    base = out0.float() if out0 is not None else torch.empty(301, F)
    ref = R.spmm(rowptr, col, x.float(), base, **rkw)
    ops = _native.ops()
    try:
        ops.set_spmm_config(variant, xcd, 128)
        out = out0.to(DEV) if out0 is not None else None
        out = K.spmm(rowptr.to(DEV), col.to(DEV), x.to(DEV), out, **kw)
    finally:
        ops.set_spmm_config(-1, -1)
    torch.testing.assert_close(out.float().cpu(), ref, atol=0.05, rtol=1e-2)


@pytest.mark.parametrize("K_VARIANT", [2, 4])
@pytest.mark.parametrize("pass_cols", [0, 64, 128])
@pytest.mark.parametrize("F", [192, 256])
def test_spmm_column_passes_bf16(pass_cols, F, K_VARIANT):
    """bf16 rows wider than ``pass_cols`` run as column passes (col_scale + beta too)."""
    from dgraph_amd import _native

    csr = _rand_csr(900, 800, 37, torch.int32, DEV, skew=True)
    x = torch.randn(800, F, device=DEV).to(torch.bfloat16)
    cs = torch.rand(800, device=DEV)
    out0 = torch.randn(900, F, device=DEV).to(torch.bfloat16)
    ref = R.spmm(csr.rowptr.cpu(), csr.col.cpu(), x.float().cpu(), out0.float().cpu(),
                 col_scale=cs.cpu(), beta=0.5)
    ops = _native.ops()
    try:
        ops.set_spmm_config(-1, -1)
        ops.set_spmm_config(K_VARIANT, 2, pass_cols)
        out = out0.clone()
        K.spmm(csr.rowptr, csr.col, x, out, col_scale=cs, beta=0.5)
    finally:
        ops.set_spmm_config(-1, -1)
    torch.testing.assert_close(out.float().cpu(), ref, atol=0.1, rtol=2e-2)


def test_spmm_deterministic():
    csr = _rand_csr(1000, 1000, 30, torch.int32, DEV, skew=True)
    x = torch.randn(1000, 128, device=DEV, dtype=torch.bfloat16)
    a = K.spmm(csr.rowptr, csr.col, x)
    b = K.spmm(csr.rowptr, csr.col, x)
    assert torch.equal(a, b)


@pytest.mark.parametrize("F", [1, 5, 8, 64, 172, 256])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_copy_rows(F, dtype):
    x = torch.randn(100, F, device=DEV).to(dtype)
    src = torch.randint(-1, 100, (77,), device=DEV)
    dst = torch.randperm(90, device=DEV)[:77]
    out = torch.zeros(90, F, device=DEV, dtype=dtype)
    K.copy_rows(x, src, dst, out)
    ref = R.copy_rows(x.cpu(), src.cpu(), dst.cpu(), torch.zeros(90, F, dtype=dtype))
    torch.testing.assert_close(out.cpu(), ref)
    g = K.gather_rows(x, src.clamp(min=0).to(torch.int32))
    torch.testing.assert_close(g.cpu(), x.cpu()[src.clamp(min=0).cpu()])


def test_copy_rows_accumulate_duplicates():
    x = torch.randn(64, 12, device=DEV)
    dst = torch.randint(0, 5, (64,), device=DEV)
    out = torch.zeros(5, 12, device=DEV)
    K.copy_rows(x, None, dst, out, accumulate=True)
    ref = torch.zeros(5, 12).index_add_(0, dst.cpu(), x.cpu())
    torch.testing.assert_close(out.cpu(), ref, atol=1e-5, rtol=1e-5)


def test_masked_gather_rows():
    x = torch.randn(10, 7, device=DEV)
    idx = torch.randint(0, 10, (20,), device=DEV)
    mask = torch.randint(0, 2, (20,), device=DEV)
    out = torch.zeros(20, 7, device=DEV)
    K.masked_gather_rows(x, idx, mask, 1, out)
    ref = R.masked_gather_rows(x.cpu(), idx.cpu(), mask.cpu(), 1, torch.zeros(20, 7))
    torch.testing.assert_close(out.cpu(), ref)


@pytest.mark.parametrize("H", [1, 3, 4, 8])
def test_edge_softmax(H):
    csr = _rand_csr(120, 120, 6, torch.int32, DEV, seed=H)
    s = torch.randn(csr.nnz, H, device=DEV) * 5
    s[:3] += 80.0  # large scores: max subtraction must keep this finite
    a = K.edge_softmax_fwd(csr.rowptr, s)
    ref = R.edge_softmax_fwd(csr.rowptr.cpu(), s.cpu())
    torch.testing.assert_close(a.cpu(), ref, atol=1e-5, rtol=1e-5)
    gr = torch.randn_like(s)
    d = K.edge_softmax_bwd(csr.rowptr, a, gr)
    dref = R.edge_softmax_bwd(csr.rowptr.cpu(), ref, gr.cpu())
    torch.testing.assert_close(d.cpu(), dref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bias_relu_pack_and_mask(dtype):
    y = torch.randn(33, 64, device=DEV).to(dtype)
    b = torch.randn(64, device=DEV)
    yc = y.clone()
    bits = torch.empty(K.mask_words(y.numel()), dtype=torch.int32, device=DEV)
    K.bias_relu_pack(y, b, bits, relu=True)
    ycpu = yc.cpu()
    bits_ref = torch.empty_like(bits.cpu())
    R.bias_relu_pack(ycpu, b.cpu(), bits_ref, True)
    torch.testing.assert_close(y.cpu(), ycpu, **_tol(dtype))
    assert torch.equal(bits.cpu(), bits_ref)
    g = torch.randn(33, 64, device=DEV).to(dtype)
    gc = g.cpu().clone()
    K.relu_mask_bwd(g, bits)
    R.relu_mask_bwd(gc, bits_ref)
    torch.testing.assert_close(g.cpu(), gc)


def test_bias_relu_pack_rejects_unaligned_rows():
    y = torch.randn(10, 172, device=DEV).to(torch.bfloat16)
    bits = torch.empty(K.mask_words(y.numel()), dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError):
        K.bias_relu_pack(y, None, bits, relu=True)


@pytest.mark.parametrize("shape", [(1000, 64), (3, 256), (777, 40), (5000, 168), (9, 8)])
def test_bias_relu_pack_shapes(shape):
    y = torch.randn(*shape, device=DEV).to(torch.bfloat16)
    yc = y.cpu().clone()
    bits = torch.empty(K.mask_words(y.numel()), dtype=torch.int32, device=DEV)
    K.bias_relu_pack(y, None, bits, relu=True)
    bref = torch.empty(bits.numel(), dtype=torch.int32)
    R.bias_relu_pack(yc, None, bref, True)
    assert torch.equal(y.cpu(), yc)
    assert torch.equal(bits.cpu(), bref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("F", [1, 5, 8, 64, 73, 172, 256])
def test_col_sum(dtype, F):
    g = torch.randn(70001, F, device=DEV).to(dtype)
    torch.testing.assert_close(K.col_sum(g).cpu(), g.float().sum(0).cpu(), atol=5e-2, rtol=1e-3)


def test_wgrad_split_k():
    from dgraph_amd.ops.dense import wgrad

    x = torch.randn(600_001, 128, device=DEV).to(torch.bfloat16)
    g = torch.randn(600_001, 96, device=DEV).to(torch.bfloat16)
    ref = x.float().t() @ g.float()
    out = wgrad(x, g, rows_per_chunk=1 << 16)
    assert out.dtype == torch.float32
    torch.testing.assert_close(out, ref, atol=0.5, rtol=1e-2)


def test_sage_stack_gpu_matches_cpu():
    from dgraph_amd.data.synthetic import SHAPES, build_partition, node_data
    from dgraph_amd.models.sage import GraphSAGE
    from dgraph_amd.parallel.dist_graph import DistGraph

    shape = SHAPES["ogbn-arxiv"].scaled(0.02)
    outs = {}
    # generate once on the CPU (device RNG streams differ), then copy
    p = build_partition(shape, 0, 1, "cpu")
    x_cpu, _, _ = node_data(shape, 0, p["offsets"], "cpu", dtype=torch.float32)
    for dev in ("cpu", DEV):
        csr = p["csr"].to(dev)
        csr.num_cols = p["L"]
        g = DistGraph(csr, p["L"], 0, symmetric=True)
        x = x_cpu.to(dev)
        torch.manual_seed(0)
        m = GraphSAGE(shape.num_features, 64, shape.num_classes, 3).to(dev)
        out = m(x, g)
        out.float().square().mean().backward()
        outs[dev] = (out.detach().cpu(), [q.grad.cpu() for q in m.parameters()])
    torch.testing.assert_close(outs[DEV][0], outs["cpu"][0], atol=1e-3, rtol=1e-3)
    for a, b in zip(outs[DEV][1], outs["cpu"][1]):
        torch.testing.assert_close(a, b, atol=1e-3, rtol=1e-2)


@pytest.mark.parametrize("F", [1, 5, 8, 16, 64, 100, 256])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
def test_pair_relu_modes(F, dtype, idx):
    csr = _rand_csr(200, 333, 9, idx, DEV, skew=True, seed=F + 7)
    P = torch.randn(200, F, device=DEV).to(dtype)
    Q = torch.randn(333, F, device=DEV).to(dtype)
    g = torch.randn(200, F, device=DEV).to(dtype)
    rc = CSR(csr.rowptr.cpu(), csr.col.cpu(), 333)
    for mode in (0, 1):
        out = K.pair_relu(csr.rowptr, csr.col, mode, P, Q, rowmul=g if mode == 1 else None)
        ref = R.pair_relu(rc.rowptr, rc.col, mode, P.cpu().float(), Q.cpu().float(),
                          rowmul=g.cpu().float() if mode == 1 else None)
        torch.testing.assert_close(out.cpu().float(), ref, **_tol(dtype))
    t = CSR(csr.rowptr, csr.col, 333).transpose()
    out = K.pair_relu(t.rowptr, t.col, 2, Q, P, gat2=g)
    tc = CSR(t.rowptr.cpu(), t.col.cpu(), 200)
    ref = R.pair_relu(tc.rowptr, tc.col, 2, Q.cpu().float(), P.cpu().float(),
                      gat2=g.cpu().float())
    torch.testing.assert_close(out.cpu().float(), ref, **_tol(dtype))


@pytest.mark.parametrize("F", [3, 8, 64, 200])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", ["none", "relu", "silu"])
def test_gather_add_act(F, dtype, act):
    E, Vs, Vd = 3000, 150, 170
    gen = torch.Generator().manual_seed(F)
    Y = torch.randn(E, F, generator=gen).to(dtype)
    P = torch.randn(Vs, F, generator=gen).to(dtype)
    Q = torch.randn(Vd, F, generator=gen).to(dtype)
    gin = torch.randn(E, F, generator=gen).to(dtype)
    src = torch.randint(0, Vs, (E,), generator=gen)
    dst = torch.randint(0, Vd, (E,), generator=gen)
    d = lambda t: t.to(DEV)  # noqa: E731
    for use_y, use_p, use_q in [(1, 1, 1), (0, 1, 1), (1, 0, 1), (1, 1, 0)]:
        kw = dict(Y=Y if use_y else None, P=P if use_p else None, src=src if use_p else None,
                  Q=Q if use_q else None, dst=dst if use_q else None)
        kwd = {k: (None if v is None else d(v)) for k, v in kw.items()}
        kwf = {k: (None if v is None else (v.float() if v.is_floating_point() else v))
               for k, v in kw.items()}
        out = K.gather_add_act(E, F, act=act, **kwd)
        ref = K.gather_add_act(E, F, act=act, **kwf)
        torch.testing.assert_close(out.cpu().float(), ref, **_tol(dtype))
        outb = K.gather_add_act(E, F, act=act, gin=d(gin), **kwd)
        refb = K.gather_add_act(E, F, act=act, gin=gin.float(), **kwf)
        torch.testing.assert_close(outb.cpu().float(), refb, **_tol(dtype))


def test_gcn_layer_gpu_matches_cpu():
    from dgraph_amd.models.gcn import GraphConvLayer

    torch.manual_seed(0)
    L, T, E, C, H = 500, 700, 6000, 32, 64
    g = torch.Generator().manual_seed(1)
    edges = torch.stack([torch.randint(0, L, (E,), generator=g),
                         torch.randint(0, T, (E,), generator=g)], 1)
    x = torch.randn(T, C, generator=g)
    layer = GraphConvLayer(2 * C, H)
    out_c = layer(x.requires_grad_(True), edges, L)
    w = torch.randn(out_c.shape, generator=g)
    (out_c * w).sum().backward()
    gx_c, gw_c = x.grad.clone(), layer.conv.weight.grad.clone()
    layer.zero_grad()
    lg = layer.to(DEV)
    xg = x.detach().to(DEV).requires_grad_(True)
    out_g = lg(xg, edges.to(DEV), L)
    (out_g * w.to(DEV)).sum().backward()
    torch.testing.assert_close(out_g.cpu(), out_c.detach(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(xg.grad.cpu(), gx_c, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(lg.conv.weight.grad.cpu(), gw_c, atol=1e-3, rtol=1e-4)


def test_gat_layer_gpu_matches_cpu():
    from dgraph_amd.data.hetero import build_relation_graph, get_vertex_offsets
    from dgraph_amd.models.rgat import CommAwareGAT

    torch.manual_seed(0)
    Ns, Nd, E, Cin, C = 900, 700, 9000, 24, 64
    g = torch.Generator().manual_seed(3)
    edges = torch.unique(torch.stack([torch.randint(0, Ns, (E,), generator=g),
                                      torch.randint(0, Nd, (E,), generator=g)]), dim=1)
    offs = {0: get_vertex_offsets(Nd, 1), 1: get_vertex_offsets(Ns, 1)}
    rel = build_relation_graph(edges, 1, 0, offs, 0, 1)
    layer = CommAwareGAT(Cin, C, heads=4, residual=True, hetero=True)
    xd = torch.randn(Nd, Cin, generator=g)
    xs = torch.randn(Ns, Cin, generator=g)
    w = torch.randn(Nd, C, generator=g)
    xdc, xsc = xd.clone().requires_grad_(True), xs.clone().requires_grad_(True)
    out_c = layer(xdc, rel, x_j=xsc)
    (out_c * w).sum().backward()
    grads_c = [p.grad.clone() for p in layer.parameters()]
    layer.zero_grad()
    lg = layer.to(DEV)
    rel = rel.to(DEV)
    xdg, xsg = xd.to(DEV).requires_grad_(True), xs.to(DEV).requires_grad_(True)
    out_g = lg(xdg, rel, x_j=xsg)
    (out_g * w.to(DEV)).sum().backward()
    torch.testing.assert_close(out_g.cpu(), out_c.detach(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(xsg.grad.cpu(), xsc.grad, atol=1e-4, rtol=1e-3)
    for a, b in zip(lg.parameters(), grads_c):
        torch.testing.assert_close(a.grad.cpu(), b, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("shape", [(1000, 128), (777, 73), (50, 512), (3, 1024), (4097, 8)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("affine,res", [(True, False), (True, True), (False, False)])
def test_layer_norm_native(shape, dtype, affine, res):
    from dgraph_amd.ops.norm import layer_norm

    g = torch.Generator().manual_seed(shape[0])
    x = (torch.randn(shape, generator=g) * 3 + 1).to(dtype)
    r = torch.randn(shape, generator=g).to(dtype) if res else None
    w = torch.randn(shape[1], generator=g) if affine else None
    b = torch.randn(shape[1], generator=g) if affine else None
    dy = torch.randn(shape, generator=g).to(dtype)
    # fp32 reference
    xr = x.float().clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True) if affine else None
    br = b.clone().requires_grad_(True) if affine else None
    yr = torch.nn.functional.layer_norm(xr, (shape[1],), wr, br, 1e-5)
    if res:
        yr = yr + r.float()
    (yr * dy.float()).sum().backward()
    xg = x.detach().to(DEV).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True) if affine else None
    bg = b.to(DEV).requires_grad_(True) if affine else None
    rg = r.to(DEV).requires_grad_(True) if res else None
    y = layer_norm(xg, wg, bg, 1e-5, rg)
    (y * dy.to(DEV)).sum().backward()
    tol = _tol(dtype)
    torch.testing.assert_close(y.float().cpu(), yr.detach(), **tol)
    torch.testing.assert_close(xg.grad.float().cpu(), xr.grad, **tol)
    if affine:
        torch.testing.assert_close(wg.grad.cpu(), wr.grad, atol=5e-2 * shape[0] ** 0.5, rtol=2e-2)
        torch.testing.assert_close(bg.grad.cpu(), br.grad, atol=5e-2 * shape[0] ** 0.5, rtol=2e-2)
    if res:
        torch.testing.assert_close(rg.grad.float().cpu(), dy.float())


@pytest.mark.parametrize("rows", [100, 5000, 300000])
def test_linear_split_k_grads(rows):
    from dgraph_amd.ops.dense import linear

    g = torch.Generator().manual_seed(rows)
    x = torch.randn(rows, 64, generator=g).to(DEV).requires_grad_(True)
    W = torch.randn(48, 64, generator=g).to(DEV).requires_grad_(True)
    b = torch.randn(48, generator=g).to(DEV).requires_grad_(True)
    dy = torch.randn(rows, 48, generator=g).to(DEV)
    y = linear(x, W, b)
    (y * dy).sum().backward()
    x2, W2, b2 = (t.detach().double().requires_grad_(True) for t in (x, W, b))
    y2 = torch.nn.functional.linear(x2, W2, b2)
    (y2 * dy.double()).sum().backward()
    torch.testing.assert_close(y.double(), y2, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(W.grad.double(), W2.grad, atol=1e-2 * rows ** 0.5 / 10, rtol=1e-3)
    torch.testing.assert_close(b.grad.double(), b2.grad, atol=1e-3 * rows ** 0.5, rtol=1e-3)
    torch.testing.assert_close(x.grad.double(), x2.grad, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("M", [1, 300, 256 * 3, 70001])
@pytest.mark.parametrize("N,K1,K2", [(256, 128, 128), (256, 256, 256), (256, 192, 192),
                                      (192, 256, 0), (128, 192, 256)])
@pytest.mark.parametrize("mode", ["relu", "plain", "cin_maskin", "cin_inplace"])
@pytest.mark.parametrize("variant", [1, 2])
def test_dual_gemm(M, N, K1, K2, mode, variant):
    """Both dual-GEMM kernels (1: column-half, B^T in LDS; 2: B-stationary in VGPRs, A
    streamed once through LDS) against an fp32 reference of the same op."""
    from dgraph_amd.ops.dense import dual_gemm, tile32_mask_words

    from dgraph_amd import _native

    ops = _native.ops()
    ops.set_dual_gemm_variant(variant)
    try:
        _dual_gemm_case(M, N, K1, K2, mode)
    finally:
        ops.set_dual_gemm_variant(2)


def _dual_gemm_case(M, N, K1, K2, mode):
    from dgraph_amd.ops.dense import dual_gemm, tile32_mask_words

    g = torch.Generator().manual_seed(M + N + K1)
    A1 = torch.randn(M, K1, generator=g).to(torch.bfloat16)
    B1 = (torch.randn(K1, N, generator=g) / K1 ** 0.5).to(torch.bfloat16)
    A2 = torch.randn(M, K2, generator=g).to(torch.bfloat16) if K2 else None
    B2 = (torch.randn(K2, N, generator=g) / K2 ** 0.5).to(torch.bfloat16) if K2 else None
    bias = torch.randn(N, generator=g)
    ref = A1.float() @ B1.float() + bias
    if K2:
        ref += A2.float() @ B2.float()
    d = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    kw = dict(A2=d(A2), B2t=None if B2 is None else d(B2.t().contiguous()), bias=d(bias))
    words = tile32_mask_words(M, N)
    if mode == "relu":
        mo = torch.zeros(words, dtype=torch.int64, device=DEV)
        out = dual_gemm(d(A1), d(B1.t().contiguous()), relu=True, mask_out=mo, **kw)
        keep = ref > 0
        torch.testing.assert_close(out.float().cpu(), torch.where(keep, ref, 0.0),
                                   atol=3e-2, rtol=2e-2)
        dec = R.tile32_decode(mo, M, N)
        # rows close to 0 may flip in bf16: compare where |ref| is not tiny
        sure = ref.abs() > 1e-2
        assert torch.equal(dec[sure], keep[sure])
        assert torch.equal(R.tile32_encode(dec), mo.cpu()[:R.tile32_encode(dec).numel()])
    elif mode == "plain":
        out = dual_gemm(d(A1), d(B1.t().contiguous()), **kw)
        torch.testing.assert_close(out.float().cpu(), ref, atol=3e-2, rtol=2e-2)
    elif mode == "cin_inplace":
        # the SAGE project-first output layer: out = A1 B1 + bias + out (cin aliases out)
        cin = torch.randn(M, N, generator=g).to(torch.bfloat16)
        buf = d(cin).clone()
        out = dual_gemm(d(A1), d(B1.t().contiguous()), cin=buf, out=buf, **kw)
        assert out.data_ptr() == buf.data_ptr()
        torch.testing.assert_close(out.float().cpu(), ref + cin.float(), atol=3e-2, rtol=2e-2)
    else:
        cin = torch.randn(M, N, generator=g).to(torch.bfloat16)
        keep = torch.rand(M, N, generator=g) > 0.4
        mi = R.tile32_encode(keep).to(DEV)
        out = dual_gemm(d(A1), d(B1.t().contiguous()), cin=d(cin), mask_in=mi, **kw)
        exp = torch.where(keep, ref + cin.float(), 0.0)
        torch.testing.assert_close(out.float().cpu(), exp, atol=3e-2, rtol=2e-2)


def test_tile32_roundtrip_cpu():
    g = torch.Generator().manual_seed(0)
    keep = torch.rand(333, 192, generator=g) > 0.5
    assert torch.equal(R.tile32_decode(R.tile32_encode(keep), 333, 192), keep)


def test_sage_stack_fused_dual_gemm_matches_unfused(monkeypatch):
    """bf16 3-layer SAGE (hidden 256, 172 classes: every combine on the MFMA dual GEMM,
    ReLU masks in the tile32 layout) vs the same model on the library GEMM path."""
    import dgraph_amd.models.sage as S
    from dgraph_amd.data.synthetic import SHAPES, build_partition, node_data
    from dgraph_amd.parallel.dist_graph import DistGraph

    shape = SHAPES["ogbn-products"].scaled(0.01)
    p = build_partition(shape, 0, 1, "cpu")
    x_cpu, _, tr = node_data(shape, 0, p["offsets"], "cpu", dtype=torch.float32)
    csr = p["csr"].to(DEV)
    csr.num_cols = p["L"]
    g = DistGraph(csr, p["L"], 0, symmetric=True)
    x = torch.nn.functional.pad(x_cpu, (0, 128 - x_cpu.shape[1])).to(DEV).to(torch.bfloat16)
    rows = torch.nonzero(tr).squeeze(1).to(DEV)
    res = {}
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(S, "_fusable", lambda *a, **k: False)
        calls = []
        orig = S.dual_gemm
        monkeypatch.setattr(S, "dual_gemm", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
        torch.manual_seed(0)
        m = S.GraphSAGE(128, 256, 172, 3).to(DEV)
        out = m(x, g, out_rows=rows)
        loss = out.float().square().mean()
        loss.backward()
        res[fused] = (out.float().cpu(), [q.grad.cpu() for q in m.parameters()], len(calls))
    # 3 full-row forward combines (the output layer is computed for every vertex) + the
    # project-first output layer's projection + 2 backward input-gradient combines
    assert res[True][2] == 6 and res[False][2] == 0
    torch.testing.assert_close(res[True][0], res[False][0], atol=5e-2, rtol=5e-2)
    for a, b in zip(res[True][1], res[False][1]):
        rel = (a - b).norm() / b.norm().clamp_min(1e-12)
        assert rel < 3e-2, float(rel)


@pytest.mark.parametrize("F,scratch_cols", [(256, 128), (192, 70), (128, 500)])
def test_aggregate_T_prescaled_matches_weighted(F, scratch_cols):
    """DistGraph.aggregate_T with a scratch slot (column slices pre-scaled, unweighted
    SpMM) equals the weighted-kernel path."""
    from dgraph_amd.parallel.dist_graph import DistGraph

    csr = _rand_csr(3000, 3000, 20, torch.int32, DEV, skew=True, seed=F)
    g = DistGraph(csr, 3000, 0)
    x = torch.randn(3000, F, device=DEV).to(torch.bfloat16)
    ref = g.aggregate_T(x)
    scratch = torch.empty(3000 * scratch_cols, dtype=torch.bfloat16, device=DEV)
    out = g.aggregate_T(x, scratch=scratch)
    torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)


def test_aggregate_T_rows_matches_dense():
    """The output-layer path: aggregate_T of a gradient that is zero off ``rows``."""
    from dgraph_amd.parallel.dist_graph import DistGraph

    csr = _rand_csr(2000, 2000, 15, torch.int32, DEV, seed=3)
    g = DistGraph(csr, 2000, 0)
    rows = torch.randperm(2000, device=DEV)[:150].sort().values
    gr = torch.randn(150, 192, device=DEV).to(torch.bfloat16)
    dense = torch.zeros(2000, 192, device=DEV, dtype=torch.bfloat16)
    dense[rows] = gr
    ref = g.aggregate_T(dense)
    out = g.aggregate_T_rows(gr, rows)
    torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("F,c0,w", [(256, 128, 128), (192, 64, 128), (64, 0, 64), (40, 8, 24)])
def test_row_scale_cols(dtype, F, c0, w):
    """Native column-slice row scale vs the fp32 PyTorch reference."""
    g = torch.randn(50_003, F, device=DEV).to(dtype)
    s = torch.rand(50_003, device=DEV) + 0.1
    out = torch.empty(50_003, w, device=DEV, dtype=dtype)
    K.row_scale_cols(g[:, c0:c0 + w], s, out)
    ref = (g[:, c0:c0 + w].float() * s.unsqueeze(1)).to(dtype)
    torch.testing.assert_close(out.float(), ref.float(), atol=0, rtol=0)


@pytest.mark.parametrize("L", [(1 << 23) - 777, (1 << 23) + 12345, 300_001])
@pytest.mark.parametrize("K,N", [(256, 128), (128, 256), (64, 64)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_wgrad_matches_fp32_reference(L, K, N, dtype):
    """Split-K batched weight gradient (dense.wgrad) vs ``x.float().t() @ g.float()``:
    just below / above the 2^23-row chunking switch of the linear layers, a remainder
    tail (L not a multiple of the chunk), the swapped K < N order, bf16 and fp32."""
    from dgraph_amd.ops.dense import _auto_rows_per_chunk, release_workspace, wgrad

    gen = torch.Generator(device="cuda").manual_seed(L + K)
    x = torch.randn(L, K, device="cuda", generator=gen).to(dtype)
    g = torch.randn(L, N, device="cuda", generator=gen).to(dtype)
    ref = x.double().t() @ g.double()
    for rpc in (0, _auto_rows_per_chunk(L)):
        out = wgrad(x, g, rpc)
        assert out.dtype == torch.float32 and out.shape == (K, N)
        # sums over L ~ 1e7 products: compare on the scale of sqrt(L)
        torch.testing.assert_close(out.double(), ref, atol=2e-3 * L ** 0.5, rtol=1e-3)
    release_workspace()
