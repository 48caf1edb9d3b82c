"""Halo recomputation on the GPU (parallel/halo_recompute.py): the fused bf16 path (MFMA
dual GEMMs with the first layer's 1-bit ReLU masks split at the padded owned/halo row
boundary, extended workspace slots) tracks the unfused fp32 path on the same inputs.

One rank of a 2-way partition runs alone with a loopback exchange (bench.py
--rehearse-world), so both runs see identical (loopback) halo data. The unfused path
itself equals W=1 training at W = 2, 4, 8 (tests/test_bench_path.py, gloo)."""
import argparse
import types

import pytest
import torch

pytestmark = pytest.mark.gpu


def _args(**kw):
    a = argparse.Namespace(shape="ogbn-papers100M", scale=2e-4, hidden=256, layers=3,
                           lr=3e-3, dtype="bf16", global_frac=0.05, window=256, seed=0,
                           no_overlap=False, rehearse_world=2, rehearse_rank=1,
                           halo_recompute="on", cuda_graph=False, executor="stack")
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _run(dtype, recompute="on", steps=4):
    import bench

    comm = types.SimpleNamespace(get_rank=lambda: 0, get_world_size=lambda: 1, group=None)
    dev = torch.device("cuda", 0)
    job = bench.Job(_args(halo_recompute=recompute), comm, dev, 0.05, dtype)
    assert job.fused is None, "the layer-stack path (the one with halo recomputation)"
    assert job.recompute == (recompute == "on")
    losses = [float(job.step(False).detach()) for _ in range(steps)]
    torch.cuda.synchronize()
    rc = job.graph.recompute if job.recompute else None
    info = (job.L, job.H, rc.L1 if rc else None)
    job.free()
    return torch.tensor(losses), info


def test_recompute_fused_bf16_tracks_unfused_fp32():
    from dgraph_amd import _native

    assert _native.load(), "native library missing"
    l16, info = _run(torch.bfloat16)
    l32, _ = _run(torch.float32)
    L, H, L1 = info
    assert H > 0 and L1 == (L + 255) // 256 * 256 + H
    assert torch.isfinite(l16).all() and torch.isfinite(l32).all()
    rel = (l16 - l32).abs() / l32.abs()
    assert float(rel.max()) < 3e-2, (l16.tolist(), l32.tolist())


def test_recompute_off_still_runs():
    l, _ = _run(torch.bfloat16, recompute="off", steps=2)
    assert torch.isfinite(l).all()
