"""Dense helpers for tall-skinny GNN shapes (rows = vertices, up to 10^8).

* :func:`wgrad` — weight gradient ``x^T g`` ([L,K]^T [L,N], L ~ 1e8, K,N <= 256) with an
  fp32 result. A plain GEMM call gives hipBLASLt a 256x256 output = 16 tiles for 256 CUs
  (79 ms per call on MI355X at L = 111M, profiles/); here the rows are cut into chunks
  and run as one batched GEMM (split-K over the batch), then the fp32 partial products
  are summed (deterministic, fixed order).
* :func:`col_sum_f32` — bias gradient via the native column-sum kernel.
"""
from __future__ import annotations

import torch

from . import kernels as K


def mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b`` with an fp32 result (bf16 operands, fp32 accumulate)."""
    if a.is_cuda and a.dtype != torch.float32:
        try:
            return torch.mm(a, b, out_dtype=torch.float32)
        except (RuntimeError, TypeError):
            pass
    return torch.mm(a, b).float()


def _bmm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if a.is_cuda and a.dtype != torch.float32:
        try:
            return torch.bmm(a, b, out_dtype=torch.float32)
        except (RuntimeError, TypeError):
            pass
    return torch.bmm(a, b).float()


def wgrad(x: torch.Tensor, g: torch.Tensor, rows_per_chunk: int = 1 << 18) -> torch.Tensor:
    """``x^T @ g`` in fp32 for tall ``x [L, K]``, ``g [L, N]`` (row-contiguous)."""
    L = x.shape[0]
    if L == 0:
        return torch.zeros(x.shape[1], g.shape[1], dtype=torch.float32, device=x.device)
    nb = L // rows_per_chunk
    if not x.is_cuda or nb < 2 or not (x.is_contiguous() and g.is_contiguous()):
        return mm_f32(x.t(), g)
    Lm = nb * rows_per_chunk
    xb = x[:Lm].view(nb, rows_per_chunk, x.shape[1]).transpose(1, 2)
    gb = g[:Lm].view(nb, rows_per_chunk, g.shape[1])
    out = _bmm_f32(xb, gb).sum(0)
    if Lm < L:
        out += mm_f32(x[Lm:].t(), g[Lm:])
    return out


def col_sum_f32(g: torch.Tensor) -> torch.Tensor:
    """fp32 column sums without an fp32 copy of ``g``."""
    return K.col_sum(g)
