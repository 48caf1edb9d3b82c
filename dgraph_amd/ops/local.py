"""Drop-in replacements of the reference's ``torch_local`` extension functions
(DGraph/distributed/csrc/torch_local_kernels.cu:28-254, bound at
torch_local_bindings.cpp:20-26), executed by this library's HIP kernels.

Signatures and ``[B, rows, F]`` layouts match the reference. Differences: any float dtype
(fp32/bf16) instead of fp32 only; launches on the current stream (the reference used the
legacy default stream); ``local_masked_scatter`` is a plain scatter-add (the reference
baked a ReLU into it, D7/K5); duplicate destinations in ``*_scatter_add_gather`` are
accumulated with fp32 atomics (bf16 outputs accumulate through an fp32 temporary).
"""
from __future__ import annotations

import torch

from . import kernels as K


def _b(t: torch.Tensor) -> torch.Tensor:
    return t.reshape(-1, t.shape[-2], t.shape[-1]) if t.dim() >= 2 else t


def local_masked_gather(input, indices, rank_local_placement, output, num_batches,
                        num_values_rows, num_cols, num_output_rows, local_rank):
    """``output[b, r] = input[b, indices[r]]`` where ``rank_local_placement[r] == local_rank``."""
    idx = indices.reshape(-1).long()
    mask = rank_local_placement.reshape(-1).long()
    for b in range(int(num_batches)):
        K.masked_gather_rows(input[b], idx, mask, int(local_rank), output[b])
    return output


def local_masked_scatter(input, indices, rank_local_placement, output, num_batches,
                         num_values_rows, num_cols, num_output_rows, rank):
    """``output[b, indices[r] mod R_out] += input[b, r]`` where the placement is ``rank``."""
    idx = indices.reshape(-1).long()
    keep = rank_local_placement.reshape(-1).long() == int(rank)
    dst = torch.where(keep, torch.remainder(idx, int(num_output_rows)), torch.full_like(idx, -1))
    for b in range(int(num_batches)):
        _accumulate_rows(input[b], None, dst, output[b])
    return output


def local_masked_scatter_gather(input, src_indices, dst_indices, output, num_batches,
                                num_values_rows, num_cols, num_output_rows):
    """``output[b, dst[i]] = input[b, src[i]]``."""
    if src_indices.numel() == 0 or dst_indices.numel() == 0:
        return output
    s = src_indices.reshape(-1).long().to(input.device)
    d = dst_indices.reshape(-1).long().to(output.device)
    for b in range(int(num_batches)):
        K.copy_rows(input[b], s, d, output[b])
    return output


def local_masked_scatter_add_gather(input, src_indices, dst_indices, output, num_batches,
                                    num_values_rows, num_cols, num_output_rows):
    """``output[b, dst[i]] += input[b, src[i]]`` (duplicates accumulate)."""
    if src_indices.numel() == 0 or dst_indices.numel() == 0:
        return output
    s = src_indices.reshape(-1).long().to(input.device)
    d = dst_indices.reshape(-1).long().to(output.device)
    for b in range(int(num_batches)):
        _accumulate_rows(input[b], s, d, output[b])
    return output


def _accumulate_rows(x, src, dst, out):
    if out.dtype == torch.float32 or not out.is_cuda:
        if out.is_cuda:
            K.copy_rows(x.float() if x.dtype != torch.float32 else x, src, dst, out,
                        accumulate=True)
        else:
            vals = x if src is None else x[src]
            keep = dst >= 0
            out.index_add_(0, dst[keep], vals[keep].to(out.dtype))
        return
    tmp = out.float()
    K.copy_rows(x.float(), src, dst, tmp, accumulate=True)
    out.copy_(tmp)
