"""Rank-local helpers with the reference's ``RankLocalOps`` names and semantics
(DGraph/distributed/RankLocalOps.py:35-327), backed by the native kernels. The per-row
Python loops of the reference fallbacks (``OptimizedLocalScatterSumGather`` :172-173,
``RankLocalReNumbering`` :248-258) are vectorised.
"""
from __future__ import annotations

import torch

from ..ops import local as L


def RankLocalMaskedGather(_src, indices, rank_mapping, rank):
    """``_src[:, indices[rank_mapping == rank]]`` (``_src`` is ``[1, N, F]``)."""
    local = indices.reshape(-1)[rank_mapping.reshape(-1) == rank].long()
    return _src[:, local]


def OptimizedRankLocalMaskedGather(src, indices, rank_mapping, output, rank):
    bs = src.shape[0]
    return L.local_masked_gather(src, indices.reshape(-1), rank_mapping.reshape(-1), output,
                                 bs, src.shape[1], src.shape[-1], output.shape[1], rank)


def OptimizedLocalScatterGather(src, src_indices, dst_indices, output):
    """``output[:, dst[i]] = src[:, src[i]]``."""
    return L.local_masked_scatter_gather(src, src_indices, dst_indices, output, src.shape[0],
                                         src_indices.numel(), src.shape[-1], output.shape[1])


def OptimizedLocalScatterSumGather(src, src_indices, dst_indices, output):
    """``output[:, dst[i]] += src[:, src[i]]``."""
    return L.local_masked_scatter_add_gather(src, src_indices, dst_indices, output,
                                             src.shape[0], src_indices.numel(), src.shape[-1],
                                             output.shape[1])


def OutOfPlaceRankLocalMaskedGather(_src, indices, rank_mapping, rank):
    local = indices.reshape(-1)[rank_mapping.reshape(-1) == rank].long()
    return _src[local]


def RankLocalMaskedScatter(_src, _output, local_indices_slice, local_dest_ranks, rank):
    """``_output[:, idx mod R] += _src[:, r]`` for rows whose destination is ``rank``."""
    m = local_dest_ranks.reshape(-1) == rank
    if bool(m.any()):
        idx = local_indices_slice.reshape(-1)[m].long() % _output.shape[1]
        _output[0].index_add_(0, idx, _src[0][m].to(_output.dtype))
    return _output


def RankLocalReNumbering(_indices):
    unique, inverse = torch.unique(_indices, return_inverse=True)
    return inverse, unique


def RankLocalRenumberingWithMapping(_indices, rank_mapping):
    unique, inverse = torch.unique(_indices, return_inverse=True)
    rank_mapping = rank_mapping.to(_indices.device)
    um = torch.zeros_like(unique, dtype=rank_mapping.dtype)
    um.scatter_(0, inverse.reshape(-1), rank_mapping.reshape(-1))
    return inverse, unique, um


def RankLocalGather(_src, indices, rank_mapping, rank):
    local = indices.reshape(-1)[rank_mapping.reshape(-1) == rank].long()
    return _src[local]


def LocalAggregateWithRemapping(global_data, global_indices, global_mapping, num_features,
                                device):
    """Pre-aggregate rows sharing an index (I4) and return the owner of each unique row."""
    inverse, unique, new_mapping = RankLocalRenumberingWithMapping(global_indices, global_mapping)
    out = torch.zeros(1, unique.numel(), num_features, dtype=global_data.dtype, device=device)
    out[0].index_add_(0, inverse.reshape(-1).to(device), global_data.reshape(-1, num_features))
    return out, new_mapping
