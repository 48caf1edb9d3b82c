#!/usr/bin/env python3
"""Static vs dynamic (work-counter) scheduling of the persistent fp32 GEMM / weight-gradient
kernels, alone and next to a kernel of another stream that holds CUs for the whole run —
what RCCL's all-to-all kernels do during a halo exchange (modelled here by ``link_delay``
waves, one per occupied CU).

    python benchmarks/bench_sched_f32.py [--rows 1438388] [--occupy 0,1,8,32]
"""
import argparse
import json
import os
import statistics
import sys

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1438388)  # the W=1 headline's chunk rows
    ap.add_argument("--occupy", default="0,1,8,32")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from dgraph_amd import _native
    from dgraph_amd.ops import f32 as F32

    _native.load()
    ops = _native.ops()
    dev = torch.device("cuda", 0)
    M = a.rows
    A1 = torch.randn(M, 256, device=dev)
    A2 = torch.randn(M, 256, device=dev)
    B1 = torch.randn(256, 256, device=dev) / 16
    B2 = torch.randn(256, 256, device=dev) / 16
    bias = torch.randn(256, device=dev)
    out = torch.empty(M, 256, device=dev)
    G = torch.randn(M, 256, device=dev)
    acc = F32.WgradAcc(256, 256, dev)
    side = torch.cuda.Stream(dev)

    def gemm():
        F32.gemm_f32(A1, B1, A2, B2, bias=bias, relu=True, out=out)

    def wgrad():
        acc.reset()
        acc.add(A1, G)
        acc.result()

    res = {}
    for name, fn in (("gemm_K512_N256", gemm), ("wgrad_256x256", wgrad)):
        for occ in [int(v) for v in a.occupy.split(",")]:
            for dyn in (0, 1):
                ops.set_f32_sched(-1, dyn)
                fn()
                torch.cuda.synchronize()
                ts = []
                for _ in range(a.reps):
                    if occ:
                        # occ single-wave blocks spinning 200 ms on the side stream, started
                        # before the timed kernel (each holds a CU the GEMM block needs)
                        with torch.cuda.stream(side):
                            ops.link_delay(200_000.0, 0, occ)
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(
                        enable_timing=True)
                    s.record()
                    fn()
                    e.record()
                    torch.cuda.synchronize()
                    ts.append(s.elapsed_time(e))
                ms = statistics.median(ts)
                res[f"{name}_occ{occ}_{'dyn' if dyn else 'static'}"] = round(ms, 3)
                print(f"{name} occupied={occ} {'dynamic' if dyn else 'static '}: {ms:.3f} ms",
                      flush=True)
    ops.set_f32_sched(-1, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
