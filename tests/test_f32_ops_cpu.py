"""CPU references of the fp32 ops (dgraph_amd.ops.f32) against dense definitions; these
references are what the gloo multi-process tests of the fused executor run."""
import torch

from dgraph_amd.ops import f32 as F32


def test_cpu_gemm_wgrad_bits():
    g = torch.Generator().manual_seed(0)
    A1, A2 = torch.randn(50, 32, generator=g), torch.randn(50, 32, generator=g)
    B1, B2 = torch.randn(32, 64, generator=g), torch.randn(32, 64, generator=g)
    out = F32.gemm_f32(A1, B1, A2, B2, bias=torch.ones(64), relu=True)
    torch.testing.assert_close(out, torch.relu(A1 @ B1 + A2 @ B2 + 1), atol=1e-4, rtol=1e-5)
    acc = F32.WgradAcc(64, 64, "cpu")
    acc.add(A1, out, A2)
    acc.add(A1[:10], out[:10], A2[:10])
    ref = torch.cat([A1, A2], 1).t() @ out + torch.cat([A1[:10], A2[:10]], 1).t() @ out[:10]
    torch.testing.assert_close(acc.result(), ref, atol=1e-3, rtol=1e-5)
    h = torch.randn(20, 64, generator=g)
    bits = F32.row_keep_bits(h)
    gg = torch.randn(20, 64, generator=g)
    torch.testing.assert_close(F32.apply_keep_bits(gg.clone(), bits),
                               torch.where(h > 0, gg, torch.zeros_like(gg)))


def test_cpu_spmm_col_map():
    rp = torch.tensor([0, 2, 3, 3, 5])
    col = torch.tensor([0, 2, 1, 3, 0], dtype=torch.int32)
    cmap = torch.tensor([1, -1, 0, -1], dtype=torch.int32)
    xc = torch.tensor([[1.0, 2.0], [10.0, 20.0]])
    out = F32.spmm_f32(rp, col, xc, col_map=cmap)
    torch.testing.assert_close(out, torch.tensor([[11.0, 22.0], [0, 0], [0, 0], [10, 20]]))
