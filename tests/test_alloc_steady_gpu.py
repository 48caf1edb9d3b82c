"""Steady-state allocator behaviour of the bench step (VERDICT r2 "stop relying on allocator
luck"): after warm-up, a training step must not call hipMalloc/hipFree (the caching
allocator's ``num_device_alloc`` / ``num_device_free`` counters stay constant), must not hit
an allocation retry (a failed hipMalloc that made the allocator release its cache), and the
reserved segment count must not grow. Covers the fp32 fused executor (the headline) and the
bf16 layer-stack path, on the scaled papers100M shape.
"""
import argparse
import types

import pytest
import torch

pytestmark = pytest.mark.gpu


def _args(**kw):
    a = argparse.Namespace(shape="ogbn-papers100M", scale=2e-4, hidden=256, layers=3, lr=1e-2,
                           dtype="fp32", global_frac=0.05, window=256, seed=0,
                           no_overlap=False, rehearse_world=0, rehearse_rank=0,
                           halo_recompute="off", executor="auto", cuda_graph=False)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _counters():
    s = torch.cuda.memory_stats()
    return {k: s.get(k, 0) for k in ("num_device_alloc", "num_device_free",
                                     "num_alloc_retries", "segment.all.current")}


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_steady_state_step_does_not_allocate(dt):
    import bench

    comm = types.SimpleNamespace(get_rank=lambda: 0, get_world_size=lambda: 1, group=None)
    dtype = torch.float32 if dt == "fp32" else torch.bfloat16
    job = bench.Job(_args(dtype=dt), comm, torch.device("cuda", 0), 0.05, dtype)
    if dt == "fp32":
        assert job.fused is not None
    try:
        for _ in range(2):  # warm-up: first-touch workspaces, autotuned configs
            job.step(False)
        torch.cuda.synchronize()
        before = _counters()
        for _ in range(3):
            job.step(False)
        torch.cuda.synchronize()
        after = _counters()
        assert after == before, (before, after)
    finally:
        job.free()
        torch.cuda.synchronize()
