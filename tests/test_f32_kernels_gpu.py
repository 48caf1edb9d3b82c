"""fp32 (reference-precision) kernels vs fp64 PyTorch references of the same op:
row-group SpMM (row lists, column maps, row maps, beta), MFMA f32 dual GEMM (every N,
split K, bias/cin/gate/ReLU, A-row gather, output-row scatter), split-M weight gradient
(accumulated over calls), keep-bit masks; hub-row splitting at odd widths.
"""
import pytest
import torch

from dgraph_amd.ops import f32 as F32
from dgraph_amd.ops import kernels as K
from dgraph_amd.ops import reference as R
from dgraph_amd.ops.csr import CSR

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _csr(R_, C, avg, seed, idx=torch.int32, hub=0):
    g = torch.Generator().manual_seed(seed)
    deg = torch.poisson(torch.full((R_,), float(avg)), generator=g).long()
    deg[R_ // 3] = 0
    if hub:
        deg[1] = hub
    rp = torch.zeros(R_ + 1, dtype=torch.long)
    rp[1:] = torch.cumsum(deg, 0)
    col = torch.randint(0, C, (int(rp[-1]),), generator=g)
    return rp.to(DEV), col.to(idx).to(DEV)


@pytest.mark.parametrize("F", [4, 32, 64, 128, 176, 256, 260])
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
def test_spmm_f32_rowgroup_vs_fp64(F, idx):
    rp, col = _csr(517, 300, 9, F, idx, hub=700)
    g = torch.Generator().manual_seed(F + 1)
    x = torch.randn(300, F, generator=g).to(DEV)
    rs = torch.rand(517, generator=g).to(DEV)
    cs = torch.rand(300, generator=g).to(DEV)
    out = K.spmm(rp, col, x, row_scale=rs, col_scale=cs)
    ref = R.spmm(rp.cpu(), col.cpu(), x.double().cpu(), torch.empty(517, F, dtype=torch.float64),
                 None, cs.cpu(), rs.cpu())
    torch.testing.assert_close(out.double().cpu(), ref, atol=2e-5, rtol=1e-5)
    # bitwise run-to-run identical (fixed order per row)
    out2 = K.spmm(rp, col, x, row_scale=rs, col_scale=cs)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("F,pc", [(32, 64), (128, 64), (256, 64), (256, 256), (256, 128)])
@pytest.mark.parametrize("frac", [0.05, 0.2, 0.9])
def test_spmm_f32_col_map_compaction(F, pc, frac):
    """Column-mapped aggregation with most entries unmapped: the kernel compacts each
    chunk's mapped entries (ballot + rank) before gathering; every lane-group width
    (8/16/32/64 lanes per row) and rows longer than one chunk, vs the CPU reference."""
    rp, col = _csr(3000, 2000, 70, 7)
    g = torch.Generator().manual_seed(int(frac * 100) + F + pc)
    nk = max(1, int(2000 * frac))
    keep = torch.randperm(2000, generator=g)[:nk].sort().values
    cmap = torch.full((2000,), -1, dtype=torch.int32)
    cmap[keep] = torch.arange(nk, dtype=torch.int32)
    xc = torch.randn(nk, F, generator=g)
    rs = torch.rand(3000, generator=g)
    ref = torch.zeros(3000, F)
    F32.spmm_f32(rp.cpu(), col.cpu(), xc, ref, row_scale=rs, col_map=cmap)
    out = torch.zeros(3000, F, device=DEV)
    F32.spmm_f32(rp, col, xc.to(DEV), out, row_scale=rs.to(DEV), col_map=cmap.to(DEV),
                 pass_cols=pc)
    torch.testing.assert_close(out.cpu(), ref, atol=2e-5, rtol=1e-5)
    out2 = torch.zeros_like(out)
    F32.spmm_f32(rp, col, xc.to(DEV), out2, row_scale=rs.to(DEV), col_map=cmap.to(DEV),
                 pass_cols=pc)
    assert torch.equal(out, out2)


def test_spmm_f32_ex_row_ids_col_map_row_map_beta():
    rp, col = _csr(400, 350, 11, 3)
    g = torch.Generator().manual_seed(5)
    F = 256
    # x is a row-compacted operand: 350 columns, 120 of them stored
    keep = torch.randperm(350, generator=g)[:120].sort().values
    cmap = torch.full((350,), -1, dtype=torch.int32)
    cmap[keep] = torch.arange(120, dtype=torch.int32)
    xc = torch.randn(120, F, generator=g)
    rows = torch.randperm(400, generator=g)[:150].sort().values
    rmap = torch.randperm(300, generator=g)[:150]
    rs = torch.rand(300, generator=g)
    base = torch.randn(300, F, generator=g)
    ref = base.clone()
    F32.spmm_f32(rp.cpu(), col.cpu(), xc, ref, row_scale=rs, col_map=cmap, row_ids=rows,
                 beta=0.5, row_map=rmap)
    out = base.to(DEV)
    F32.spmm_f32(rp, col, xc.to(DEV), out, row_scale=rs.to(DEV), col_map=cmap.to(DEV),
                 row_ids=rows.to(DEV), beta=0.5, row_map=rmap.to(DEV))
    torch.testing.assert_close(out.cpu(), ref, atol=2e-5, rtol=1e-5)
    # CPU oracle against the dense definition
    A = torch.zeros(400, 350, dtype=torch.float64)
    r_ids = torch.repeat_interleave(torch.arange(400), (rp[1:] - rp[:-1]).cpu())
    A.index_put_((r_ids, col.cpu().long()), torch.ones(r_ids.numel(), dtype=torch.float64),
                 accumulate=True)
    xf = torch.zeros(350, F, dtype=torch.float64)
    xf[keep] = xc.double()
    dense = (A[rows] @ xf) * rs.double()[rmap].unsqueeze(1) + 0.5 * base.double()[rmap]
    torch.testing.assert_close(ref[rmap].double(), dense, atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("N", [64, 128, 176, 192, 256])
@pytest.mark.parametrize("K1,K2", [(128, 128), (256, 256), (256, 0), (128, 0)])
def test_gemm_f32_dual_vs_fp64(N, K1, K2):
    g = torch.Generator().manual_seed(N + K1 + K2)
    M = 1000  # not a multiple of the 256-row block
    A1 = torch.randn(M, K1, generator=g)
    B1 = torch.randn(K1, N, generator=g) / K1 ** 0.5
    A2 = torch.randn(M, K2, generator=g) if K2 else None
    B2 = torch.randn(K2, N, generator=g) / K2 ** 0.5 if K2 else None
    bias = torch.randn(N, generator=g)
    out = F32.gemm_f32(A1.to(DEV), B1.to(DEV), None if A2 is None else A2.to(DEV),
                       None if B2 is None else B2.to(DEV), bias=bias.to(DEV), relu=True)
    ref = A1.double() @ B1.double() + bias.double()
    if K2:
        ref = ref + A2.double() @ B2.double()
    ref = ref.clamp_min(0)
    torch.testing.assert_close(out.double().cpu(), ref, atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("N", [176, 256])
def test_gemm_f32_persistent_multi_tile(N):
    """More 256-row tiles than CUs: every persistent block walks several tiles and loads the
    next tile's first stage (gathered A1 rows, dense A2 rows) during the current one."""
    g = torch.Generator().manual_seed(21 + N)
    M = 256 * 256 * 2 + 777
    src = torch.randn(M + 5000, 128, generator=g)
    a_rows = torch.randperm(M + 5000, generator=g)[:M]
    A2 = torch.randn(M, 128, generator=g)
    B1 = torch.randn(128, N, generator=g) / 11
    B2 = torch.randn(128, N, generator=g) / 11
    bias = torch.randn(N, generator=g)
    rs = torch.rand(M, generator=g) + 0.5
    o_rows = torch.randperm(M + 100, generator=g)[:M]
    out = torch.zeros(M + 100, N).to(DEV)
    F32.gemm_f32(src.to(DEV), B1.to(DEV), A2.to(DEV), B2.to(DEV), a_rows=a_rows.to(DEV),
                 bias=bias.to(DEV), relu=True, o_rows=o_rows.to(DEV), out=out,
                 row_scale=rs.to(DEV))
    v = (src[a_rows].double() @ B1.double() + A2.double() @ B2.double()) * rs.double()[:, None]
    ref = torch.zeros(M + 100, N, dtype=torch.float64)
    ref[o_rows] = (v + bias.double()).clamp_min(0)
    torch.testing.assert_close(out.double().cpu(), ref, atol=1e-4, rtol=1e-5)


def test_gemm_f32_cin_gate_rows():
    g = torch.Generator().manual_seed(9)
    M, K1, N = 700, 256, 256
    src = torch.randn(1500, K1, generator=g)
    a_rows = torch.randperm(1500, generator=g)[:M]
    A2 = torch.randn(M, 128, generator=g)
    B1 = torch.randn(K1, N, generator=g) / 16
    B2 = torch.randn(128, N, generator=g) / 11
    o_rows = torch.randperm(900, generator=g)[:M]
    out0 = torch.randn(900, N, generator=g)
    gate = torch.randn(900, N, generator=g)
    dev = {k: v.to(DEV) for k, v in dict(src=src, a_rows=a_rows, A2=A2, B1=B1, B2=B2,
                                         o_rows=o_rows, out=out0.clone(), gate=gate).items()}
    F32.gemm_f32(dev["src"], dev["B1"], dev["A2"], dev["B2"], a_rows=dev["a_rows"],
                 cin=dev["out"], beta=0.75, gate=dev["gate"], o_rows=dev["o_rows"],
                 out=dev["out"])
    ref = out0.double().clone()
    v = src.double()[a_rows] @ B1.double() + A2.double() @ B2.double() + 0.75 * ref[o_rows]
    v = torch.where(gate[o_rows] > 0, v, torch.zeros_like(v))
    ref[o_rows] = v
    torch.testing.assert_close(dev["out"].double().cpu(), ref, atol=1e-4, rtol=1e-5)
    # CPU wrapper agrees with the same definition
    cpu_out = out0.clone()
    F32.gemm_f32(src, B1, A2, B2, a_rows=a_rows, cin=cpu_out, beta=0.75, gate=gate,
                 o_rows=o_rows, out=cpu_out)
    torch.testing.assert_close(cpu_out.double(), ref, atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("K1,K2,N", [(128, 128, 256), (256, 0, 256), (128, 0, 176),
                                     (256, 0, 128), (128, 0, 128), (128, 128, 192)])
def test_wgrad_f32_vs_fp64(K1, K2, N):
    """exact-f32 weight gradients (wgrad_f32.hip) against fp64, accumulated over two
    calls."""
    g = torch.Generator().manual_seed(K1 * 7 + N)
    M1, M2 = 5003, 777
    src = torch.randn(8000, K1, generator=g)
    rows1 = torch.randperm(8000, generator=g)[:M1]
    A2a = torch.randn(M1, K2, generator=g) if K2 else None
    G1 = torch.randn(M1, N, generator=g)
    A1b = torch.randn(M2, K1, generator=g)
    A2b = torch.randn(M2, K2, generator=g) if K2 else None
    G2 = torch.randn(M2, N, generator=g)
    acc = F32.WgradAcc(K1 + K2, N, DEV)
    acc.add(src.to(DEV), G1.to(DEV), None if A2a is None else A2a.to(DEV), rows1.to(DEV))
    acc.add(A1b.to(DEV), G2.to(DEV), None if A2b is None else A2b.to(DEV))
    out = acc.result()
    a1 = src.double()[rows1]
    if K2:
        a1 = torch.cat([a1, A2a.double()], 1)
    a2 = A1b.double() if not K2 else torch.cat([A1b.double(), A2b.double()], 1)
    ref = a1.t() @ G1.double() + a2.t() @ G2.double()
    torch.testing.assert_close(out.double().cpu(), ref, atol=2e-3, rtol=1e-5)
    # fixed block order: identical on a rerun
    acc.reset()
    acc.add(src.to(DEV), G1.to(DEV), None if A2a is None else A2a.to(DEV), rows1.to(DEV))
    acc.add(A1b.to(DEV), G2.to(DEV), None if A2b is None else A2b.to(DEV))
    assert torch.equal(out, acc.result())


def test_keep_bits_roundtrip():
    g = torch.Generator().manual_seed(3)
    h = torch.randn(500, 256, generator=g)
    rows = torch.randperm(500, generator=g)[:123]
    bits = F32.row_keep_bits(h.to(DEV), rows.to(DEV))
    bits_cpu = F32.row_keep_bits(h, rows)
    assert torch.equal(bits.cpu(), bits_cpu)
    gr = torch.randn(123, 256, generator=g)
    out = F32.apply_keep_bits(gr.to(DEV).clone(), bits)
    ref = torch.where(h[rows] > 0, gr, torch.zeros_like(gr))
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("F,dtype", [(47, torch.bfloat16), (153, torch.bfloat16),
                                     (47, torch.float32), (6, torch.bfloat16)])
def test_hub_split_odd_width(F, dtype):
    """Hub-row partials at widths that are not a multiple of the 16-B vector (ADVICE r2:
    the partials kernel used a fixed 4/2-wide vector and read/wrote past the row)."""
    rp, col = _csr(300, 280, 6, F, hub=9000)
    csr = CSR(rp, col, 280)
    sp = csr.hub_split(512)
    g = torch.Generator().manual_seed(F)
    x = torch.randn(280, F, generator=g).to(dtype).to(DEV)
    rs = torch.rand(300, generator=g).to(DEV)
    out = K.spmm(rp, col, x, row_scale=rs, split=sp)
    ref = R.spmm(rp.cpu(), col.cpu(), x.double().cpu(), torch.empty(300, F, dtype=torch.float64),
                 None, None, rs.cpu())
    tol = dict(atol=3e-2, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(out.double().cpu(), ref, **tol)


@pytest.mark.parametrize("F,pc", [(256, 256), (256, 64), (128, 128), (64, 64)])
def test_spmm_f32_col_map_two_sources(F, pc):
    """The pulled backward halo (models/sage_fused.py BWD_HALO="pull"): one column map over
    local + halo columns whose mapped index is split between the support-row operand (< nS)
    and the received halo support rows (>= nS), with beta, gate and the self term, vs the
    CPU fp64 reference and against the dense definition; bitwise run to run."""
    L, H, nS, nH = 900, 700, 260, 230
    rp, col = _csr(L, L + H, 23, 17)
    g = torch.Generator().manual_seed(F + pc)
    sk = torch.randperm(L, generator=g)[:nS].sort().values
    hk = torch.randperm(H, generator=g)[:nH].sort().values
    cmap = torch.full((L + H,), -1, dtype=torch.int32)
    cmap[sk] = torch.arange(nS, dtype=torch.int32)
    cmap[L + hk] = nS + torch.arange(nH, dtype=torch.int32)
    u = torch.randn(nS, F, generator=g)
    uh = torch.randn(nH, F, generator=g)
    v = torch.randn(nS, F, generator=g)
    gate = torch.randn(L, F, generator=g)
    base = torch.randn(L, F, generator=g) * (gate > 0)
    kw = dict(col_map=cmap, x2=uh, nsplit=nS, gate=gate, self_add=v,
              self_map=cmap[:L].contiguous(), beta=1.0)
    ref = base.clone()
    F32.spmm_f32(rp.cpu(), col.cpu(), u, ref, **kw)
    dkw = {k: (t.to(DEV) if isinstance(t, torch.Tensor) else t) for k, t in kw.items()}
    out = base.clone().to(DEV)
    F32.spmm_f32(rp, col, u.to(DEV), out, pass_cols=pc, **dkw)
    torch.testing.assert_close(out.cpu(), ref, atol=2e-5, rtol=1e-5)
    out2 = base.clone().to(DEV)
    F32.spmm_f32(rp, col, u.to(DEV), out2, pass_cols=pc, **dkw)
    assert torch.equal(out, out2)
    # dense definition: sum over mapped entries of [u; uh][cmap[c]], + self, gated, + base
    A = torch.zeros(L, L + H, dtype=torch.float64)
    r_ids = torch.repeat_interleave(torch.arange(L), (rp[1:] - rp[:-1]).cpu())
    A.index_put_((r_ids, col.cpu().long()), torch.ones(r_ids.numel(), dtype=torch.float64),
                 accumulate=True)
    xf = torch.zeros(L + H, F, dtype=torch.float64)
    xf[sk] = u.double()
    xf[L + hk] = uh.double()
    sv = torch.zeros(L, F, dtype=torch.float64)
    sv[sk] = v.double()
    dense = torch.where(gate > 0, A @ xf + sv + base.double(), torch.zeros(1, dtype=torch.float64))
    torch.testing.assert_close(out.double().cpu(), dense, atol=1e-4, rtol=1e-5)


def test_spmm_f32_self_add_gate():
    rp, col = _csr(300, 300, 7, 11)
    g = torch.Generator().manual_seed(2)
    F = 256
    u = torch.randn(90, F, generator=g)
    keep = torch.randperm(300, generator=g)[:90].sort().values
    smap = torch.full((300,), -1, dtype=torch.int32)
    smap[keep] = torch.arange(90, dtype=torch.int32)
    v = torch.randn(90, F, generator=g)
    gate = torch.randn(120, F, generator=g)
    r0, r1 = 100, 220
    ref = torch.empty(r1 - r0, F)
    F32.spmm_f32(rp.cpu()[r0:r1 + 1], col.cpu(), u, ref, col_map=smap, gate=gate,
                 self_add=v, self_map=smap, self_row0=r0)
    out = torch.empty(r1 - r0, F, device=DEV)
    F32.spmm_f32(rp[r0:r1 + 1], col, u.to(DEV), out, col_map=smap.to(DEV), gate=gate.to(DEV),
                 self_add=v.to(DEV), self_map=smap.to(DEV), self_row0=r0)
    torch.testing.assert_close(out.cpu(), ref, atol=2e-5, rtol=1e-5)
    # the self term appears exactly on the rows that are in the support
    rows = torch.arange(r0, r1)
    m = smap[rows]
    assert bool(((m >= 0) | (ref.abs().sum(1) >= 0)).all())


@pytest.mark.parametrize("C,W", [(172, 192), (47, 64), (256, 256)])
def test_xent_argmax_rows_vs_cpu(C, W):
    g = torch.Generator().manual_seed(C)
    z = torch.randn(500, 256, generator=g) * 3
    rows = torch.randperm(500, generator=g)[:150]
    y = torch.randint(0, C, (150,), generator=g)
    dz = torch.full((150, W), 7.0)
    rl = torch.zeros(150)
    F32.xent_rows(z, rows, y, 0.5, dz, rl, C)
    dzg = torch.full((150, W), 7.0, device=DEV)
    rlg = torch.zeros(150, device=DEV)
    F32.xent_rows(z.to(DEV), rows.to(DEV), y.to(DEV), 0.5, dzg, rlg, C)
    torch.testing.assert_close(dzg.cpu(), dz, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(rlg.cpu(), rl, atol=1e-5, rtol=1e-5)
    ref_loss = torch.nn.functional.cross_entropy(z[rows][:, :C].double(), y, reduction="none")
    torch.testing.assert_close(rlg.double().cpu(), ref_loss, atol=1e-5, rtol=1e-5)
    z[rows[0], 3] = z[rows[0], 5] = 1e3  # a tie: the first maximum wins (torch semantics)
    hit = torch.zeros(150, dtype=torch.uint8)
    F32.argmax_hits(z, rows, y, hit, C)
    hitg = torch.zeros(150, dtype=torch.uint8, device=DEV)
    F32.argmax_hits(z.to(DEV), rows.to(DEV), y.to(DEV), hitg, C)
    assert torch.equal(hitg.cpu(), hit)
    assert torch.equal(hit.bool(), z[rows][:, :C].argmax(1) == y)


# ---------------------------------------------------------------- wide shapes (tiled)
@pytest.mark.parametrize("N", [384, 512])
def test_gemm_f32_column_blocks_vs_fp64(N):
    """N > 256 runs as column blocks (a 512-wide hidden layer): bias, cin, gate, ReLU and
    the output row scatter per block."""
    g = torch.Generator().manual_seed(N)
    M, K1, K2 = 3000, 512, 512
    A1 = torch.randn(M, K1, generator=g)
    A2 = torch.randn(M, K2, generator=g)
    B1 = torch.randn(K1, N, generator=g) / K1 ** 0.5
    B2 = torch.randn(K2, N, generator=g) / K2 ** 0.5
    bias = torch.randn(N, generator=g)
    cin = torch.randn(M, N, generator=g)
    gate = torch.randn(M, N, generator=g)
    orows = torch.randperm(M, generator=g)
    out = cin.clone().to(DEV)
    F32.gemm_f32(A1.to(DEV), B1.to(DEV), A2.to(DEV), B2.to(DEV), bias=bias.to(DEV),
                 cin=out, beta=0.5, gate=gate.to(DEV), o_rows=orows.to(DEV), out=out)
    v = A1.double() @ B1.double() + A2.double() @ B2.double() + bias.double()
    ref = cin.double().clone()
    v = v + 0.5 * cin.double()[orows]
    v = torch.where(gate[orows] > 0, v, torch.zeros_like(v))
    ref[orows] = v
    torch.testing.assert_close(out.double().cpu(), ref, atol=2e-4, rtol=1e-5)


@pytest.mark.parametrize("K1,K2,N", [(768, 768, 256), (256, 256, 512), (320, 192, 384)])
def test_wgrad_tiles_vs_fp64(K1, K2, N):
    """[A1[rows] | A2]^T G wider than one kernel tile: K-blocks (one straddling A1 / A2 for
    K1 = 320) and N-blocks, accumulated over two calls."""
    g = torch.Generator().manual_seed(K1 + N)
    M = 4000
    src = torch.randn(6000, K1, generator=g)
    rows = torch.randperm(6000, generator=g)[:M]
    A2 = torch.randn(M, K2, generator=g)
    G = torch.randn(M, N, generator=g)
    acc = F32.WgradAcc(K1 + K2, N, DEV, colsum=True)
    half = M // 2
    acc.add(src.to(DEV), G[:half].to(DEV), A2[:half].to(DEV), rows[:half].to(DEV))
    acc.add(src.to(DEV), G[half:].to(DEV), A2[half:].to(DEV), rows[half:].to(DEV))
    out = acc.result()
    a = torch.cat([src.double()[rows], A2.double()], 1)
    ref = a.t() @ G.double()
    torch.testing.assert_close(out.double().cpu(), ref, atol=5e-3, rtol=1e-5)
    # the fused column sums (bias gradient) of the same G
    torch.testing.assert_close(acc.col_result().double().cpu(), G.double().sum(0),
                               atol=1e-3, rtol=1e-5)
    acc.reset()  # a fresh accumulation overwrites every slab it uses
    acc.add(src.to(DEV), G[:100].to(DEV), A2[:100].to(DEV), rows[:100].to(DEV))
    torch.testing.assert_close(acc.col_result().double().cpu(), G[:100].double().sum(0),
                               atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("hidden,feat,layers", [(512, 300, 3), (128, 100, 2), (384, 768, 3)])
def test_fused_wide_gpu_matches_cpu(hidden, feat, layers):
    """The fused executor at hidden 128 / 384 / 512 and wide inputs on the GPU kernels
    (tiled GEMMs and weight gradients) against the same executor on the CPU (fp64
    references of every op)."""
    from dgraph_amd.data.synthetic import (SHAPES, SPLIT_TEST, SPLIT_TRAIN, SPLIT_VALID,
                                           GraphShape, build_partition, contiguous_offsets,
                                           node_data)
    from dgraph_amd.models.sage import GraphSAGE
    from dgraph_amd.models.sage_fused import FusedSAGE
    from dgraph_amd.parallel.dist_graph import DistGraph

    base = SHAPES["ogbn-papers100M"].scaled(1e-4)
    shape = GraphShape("w", base.num_nodes, base.num_directed_edges, feat, 47, 0.2, 0.1, 0.1)
    # one graph and one data set (the generators differ per device), moved to each device
    part = build_partition(shape, 0, 1, "cpu", global_frac=0.1, window=256)
    L = part["L"]
    part["csr"].num_cols = L
    x0, y0, split0 = node_data(shape, 0, contiguous_offsets(shape.num_nodes, 1), "cpu",
                               dtype=torch.float32, return_split=True)
    res = []
    for dev in ("cpu", DEV):
        x, y, split = x0.to(dev), y0.to(dev), split0.to(dev)
        csr = part["csr"].to(dev)
        tr = torch.nonzero(split == SPLIT_TRAIN).reshape(-1)
        ev = torch.nonzero((split == SPLIT_VALID) | (split == SPLIT_TEST)).reshape(-1)
        torch.manual_seed(0)
        model = GraphSAGE(feat, hidden, 47, layers).to(dev)
        g = DistGraph(csr, L, 0, symmetric=True)
        ex = FusedSAGE(model, g, x, tr, y[tr], ev, y[ev], split[ev] == SPLIT_VALID,
                       tr.numel(), chunk_rows=2048)
        loss = ex.step()
        res.append((float(loss), [p.grad.detach().double().cpu() for p in model.parameters()],
                    ex.correct.cpu()))
    assert abs(res[0][0] - res[1][0]) < 1e-4 * max(1.0, abs(res[0][0]))
    for a, b in zip(res[0][1], res[1][1]):
        torch.testing.assert_close(b, a, atol=5e-5, rtol=2e-3)


@pytest.mark.parametrize("M,K,N", [(5000, 384, 128), (3000, 768, 512), (2000, 256, 153)])
def test_dense_linear_f32_vs_fp64(M, K, N):
    """``ops.dense.linear`` / ``linear_sum`` / ``act_linears`` at fp32 on the GPU (MFMA
    GEMM + split-M weight gradient; 153 columns on the library fallback) vs fp64 CPU."""
    from dgraph_amd.ops.act_linear import act_linears
    from dgraph_amd.ops.dense import linear, linear_sum

    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g)
    x2 = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    W2 = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    go = torch.randn(M, N, generator=g)

    def run(dev, dt, fn):
        ts = [t.to(dev, dt, copy=True).requires_grad_() for t in (x, x2, W, W2, b)]
        out = fn(*ts)
        out.backward(go.to(dev, dt))
        return [out.detach().double().cpu()] + [t.grad.double().cpu() for t in ts
                                                 if t.grad is not None]

    fns = {
        "linear": lambda a, a2, w, w2, bb: linear(a, w, bb),
        "linear_sum": lambda a, a2, w, w2, bb: linear_sum([(a, w), (a2, w2)], bb),
        "act_linears": lambda a, a2, w, w2, bb: act_linears(a, [w, w2], bb)[0]
        + act_linears(a, [w, w2], bb)[1],
    }
    for name, fn in fns.items():
        got = run(DEV, torch.float32, fn)
        ref = run("cpu", torch.float64, fn)
        assert len(got) == len(ref), name
        for a, r in zip(got, ref):
            err = float((a - r).abs().max() / r.abs().max().clamp_min(1e-6))
            assert err < 2e-5, (name, err)


# ------------------------------------------- in-place wide GEMM
@pytest.mark.parametrize("N", [384, 512])
def test_gemm_f32_column_blocks_in_place(N):
    """``out is A2`` at N > 256 (the boundary-row store / streamed halo of a 384/512-wide
    hidden layer: the aggregate rows are overwritten by the layer's output). Column block
    0 must not feed its results to block 1 as the aggregate."""
    g = torch.Generator().manual_seed(N + 3)
    M, K1 = 2000, 256
    A1 = torch.randn(M, K1, generator=g)
    agg = torch.randn(M, N, generator=g)
    B1 = torch.randn(K1, N, generator=g) / K1 ** 0.5
    B2 = torch.randn(N, N, generator=g) / N ** 0.5
    bias = torch.randn(N, generator=g)
    ref = (A1.double() @ B1.double() + agg.double() @ B2.double() + bias.double()).clamp_min(0)
    buf = agg.to(DEV)
    F32.gemm_f32(A1.to(DEV), B1.to(DEV), buf, B2.to(DEV), bias=bias.to(DEV), relu=True,
                 out=buf)
    torch.testing.assert_close(buf.double().cpu(), ref, atol=2e-4, rtol=1e-5)
    # a row-chunk view of a larger buffer (the executor's hout[r0:r1])
    big = torch.zeros(M + 300, N, device=DEV)
    big[100:100 + M] = agg.to(DEV)
    view = big[100:100 + M]
    F32.gemm_f32(A1.to(DEV), B1.to(DEV), view, B2.to(DEV), bias=bias.to(DEV), relu=True,
                 out=view)
    torch.testing.assert_close(view.double().cpu(), ref, atol=2e-4, rtol=1e-5)
    assert float(big[:100].abs().sum()) == 0 and float(big[100 + M:].abs().sum()) == 0


# ------------------------------- determinism under CU contention
def _contend(cus: int, us: float = 4000.0):
    """A link_delay kernel holding ``cus`` CUs (one wave each, the whole-CU GEMM blocks
    cannot start there) on another stream, issued before the kernel under test."""
    from dgraph_amd import _native

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        _native.ops().link_delay(float(us), 0, int(cus))
    return side


def _sched(dynamic: bool):
    from dgraph_amd import _native

    _native.ops().set_f32_sched(-1, 1 if dynamic else 0)


def _gemm_cases():
    g = torch.Generator().manual_seed(77)
    cases = []
    # many tiles, gathered A1 rows, dense A2, scattered output rows, partial last tile
    M = 256 * 256 * 2 + 777
    src = torch.randn(M + 5000, 128, generator=g)
    cases.append(dict(A1=src, B1=torch.randn(128, 256, generator=g) / 11,
                      A2=torch.randn(M, 128, generator=g), B2=torch.randn(128, 256, generator=g) / 11,
                      a_rows=torch.randperm(M + 5000, generator=g)[:M],
                      bias=torch.randn(256, generator=g), relu=True, out_rows=M))
    # N = 176, single operand, fewer tiles than CUs, partial last tile
    cases.append(dict(A1=torch.randn(5000, 256, generator=g),
                      B1=torch.randn(256, 176, generator=g) / 16, A2=None, B2=None,
                      a_rows=None, bias=None, relu=False, out_rows=5000))
    return cases


@pytest.mark.parametrize("cus", [1, 16, 64])
def test_gemm_f32_dynamic_under_contention_bitwise(cus):
    for c in _gemm_cases():
        d = {k: (v.to(DEV) if isinstance(v, torch.Tensor) else v) for k, v in c.items()}

        def run():
            out = torch.zeros(d["out_rows"], d["B1"].shape[1], device=DEV)
            F32.gemm_f32(d["A1"], d["B1"], d["A2"], d["B2"], a_rows=d["a_rows"],
                         bias=d["bias"], relu=d["relu"], out=out)
            return out

        try:
            _sched(False)
            ref = run()
            torch.cuda.synchronize()
            _sched(True)
            for _ in range(2):
                _contend(cus)
                got = run()
                torch.cuda.synchronize()
                assert torch.equal(ref, got), cus
        finally:
            _sched(True)
    # in place (out is A2, one tile width): the streamed forward's GEMM
    g = torch.Generator().manual_seed(5)
    M = 256 * 300 + 33
    A1 = torch.randn(M, 256, generator=g).to(DEV)
    agg = torch.randn(M, 256, generator=g).to(DEV)
    B1 = (torch.randn(256, 256, generator=g) / 16).to(DEV)
    B2 = (torch.randn(256, 256, generator=g) / 16).to(DEV)
    try:
        _sched(False)
        ref = agg.clone()
        F32.gemm_f32(A1, B1, ref, B2, relu=True, out=ref)
        torch.cuda.synchronize()
        _sched(True)
        got = agg.clone()
        _contend(cus)
        F32.gemm_f32(A1, B1, got, B2, relu=True, out=got)
        torch.cuda.synchronize()
        assert torch.equal(ref, got)
    finally:
        _sched(True)


@pytest.mark.parametrize("cus", [1, 16, 64])
@pytest.mark.parametrize("K1,K2,N", [(128, 128, 256), (256, 0, 176)])
def test_wgrad_f32_dynamic_under_contention_bitwise(cus, K1, K2, N):
    g = torch.Generator().manual_seed(K1 + N + cus)
    M1, M2 = 200_003, 4_321  # partial last stages, two accumulated calls
    src = torch.randn(250_000, K1, generator=g).to(DEV)
    rows = torch.randperm(250_000, generator=g)[:M1].to(DEV)
    A2a = torch.randn(M1, K2, generator=g).to(DEV) if K2 else None
    G1 = torch.randn(M1, N, generator=g).to(DEV)
    A1b = torch.randn(M2, K1, generator=g).to(DEV)
    A2b = torch.randn(M2, K2, generator=g).to(DEV) if K2 else None
    G2 = torch.randn(M2, N, generator=g).to(DEV)

    def run(contend):
        acc = F32.WgradAcc(K1 + K2, N, DEV, colsum=True)
        if contend:
            _contend(cus)
        acc.add(src, G1, A2a, rows)
        if contend:
            _contend(cus)
        acc.add(A1b, G2, A2b)
        out = acc.result()
        col = acc.col_result()
        torch.cuda.synchronize()
        return out, col

    try:
        _sched(False)
        ref, refc = run(False)
        _sched(True)
        got, gotc = run(True)
        assert torch.equal(ref, got) and torch.equal(refc, gotc)
    finally:
        _sched(True)


@pytest.mark.parametrize("cus", [1, 16, 64])
def test_spmm_f32_under_contention_bitwise(cus):
    """The row-group SpMM (fixed per-row order) with a capped persistent grid and with the
    default grid, with and without CUs held by another stream: bitwise identical."""
    from dgraph_amd import _native

    rp, col = _csr(200_000, 150_000, 12, 3, hub=5000)
    g = torch.Generator().manual_seed(cus)
    x = torch.randn(150_000, 256, generator=g).to(DEV)
    rs = torch.rand(200_000, generator=g).to(DEV)
    refs = {}
    for pc in (64, 256):  # the uncontended full-grid result of each pass width
        refs[pc] = F32.spmm_f32(rp, col, x, torch.empty(200_000, 256, device=DEV),
                                row_scale=rs, pass_cols=pc)
    torch.cuda.synchronize()
    try:
        for grid in (0, 512):
            _native.ops().set_f32_sched(grid, -1)
            for pc in (64, 256):
                _contend(cus)
                out = torch.empty_like(refs[pc])
                F32.spmm_f32(rp, col, x, out, row_scale=rs, pass_cols=pc)
                torch.cuda.synchronize()
                assert torch.equal(refs[pc], out), (grid, pc)
    finally:
        _native.ops().set_f32_sched(0, -1)


@pytest.mark.parametrize("N", [176, 256, 512])
def test_gemm_f32_fused_send_rows(N):
    """The halo pack fused into the producing GEMM (models/sage_fused.py FUSED_PACK): every
    output row is also stored at its send-buffer positions (0 to 3 per row, rows of a
    sub-range as the boundary chunks pass them); the send rows equal the output rows
    bitwise and nothing else of the send buffer is written. N = 512 runs as column blocks."""
    g = torch.Generator().manual_seed(N)
    L, M0, M1, K = 1500, 300, 1300, 256
    x = torch.randn(L, K, generator=g)
    W = torch.randn(K, N, generator=g) / 16
    bias = torch.randn(N, generator=g)
    cnt = torch.randint(0, 4, (L,), generator=g)
    cnt[:M0] = 0  # (interior rows: sent to nobody)
    ptr = torch.zeros(L + 1, dtype=torch.long)
    ptr[1:] = torch.cumsum(cnt, 0)
    n_send = int(ptr[-1])
    pos = torch.randperm(n_send, generator=g).to(torch.int32)
    send = torch.full((n_send + 7, N), -7.0).to(DEV)
    out = torch.zeros(L, N).to(DEV)
    F32.gemm_f32(x[M0:M1].to(DEV), W.to(DEV), bias=bias.to(DEV), relu=True,
                 out=out[M0:M1], send=(send, ptr[M0:M1 + 1].to(DEV), pos.to(DEV)))
    ref = (x[M0:M1].double() @ W.double() + bias.double()).clamp_min(0)
    torch.testing.assert_close(out[M0:M1].double().cpu(), ref, atol=1e-4, rtol=1e-5)
    so, oc = send.cpu(), out.cpu()
    written = torch.zeros(n_send + 7, dtype=torch.bool)
    for r in range(M0, M1):
        for q in range(int(ptr[r]), int(ptr[r + 1])):
            assert torch.equal(so[int(pos[q])], oc[r]), (r, q)
            written[int(pos[q])] = True
    assert bool((so[~written] == -7.0).all())


@pytest.mark.parametrize("F,pc", [(256, 64), (256, 256), (128, 128)])
def test_spmm_f32_keep_bits(F, pc):
    """The 1-bit ReLU mask in the SpMM epilogue (models/sage_fused.py output-layer
    backward): columns whose keep bit is clear are zeroed, every column pass reading its own
    bits; with a row map and beta = 1 too. Against the CPU fp64 reference."""
    rp, col = _csr(700, 500, 13, 5 + F)
    g = torch.Generator().manual_seed(F + pc)
    x = torch.randn(500, F, generator=g)
    h = torch.randn(900, F, generator=g)
    bits = F32.row_keep_bits(h)  # [900, F/32]
    rmap = torch.randperm(900, generator=g)[:700]
    base = torch.randn(900, F, generator=g)
    for kw in (dict(), dict(row_map=rmap, beta=1.0)):
        ref = base.clone()
        F32.spmm_f32(rp.cpu(), col.cpu(), x, ref, keep_bits=bits,
                     **{k: v for k, v in kw.items()})
        out = base.clone().to(DEV)
        F32.spmm_f32(rp, col, x.to(DEV), out, keep_bits=bits.to(DEV), pass_cols=pc,
                     **{k: (v.to(DEV) if isinstance(v, torch.Tensor) else v)
                        for k, v in kw.items()})
        torch.testing.assert_close(out.cpu(), ref, atol=2e-5, rtol=1e-5)
        o = rmap if "row_map" in kw else torch.arange(700)
        assert bool((out.cpu()[o][h[o] <= 0] == 0).all())
