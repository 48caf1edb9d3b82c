"""LayerNorm kernel bandwidth at the GraphCast shapes (csrc/kernels/layernorm.hip).

Rows: processor mesh edges (655,320), grid nodes (1,038,240), encoder/decoder edges
(~1.6 M / ~3.1 M); F = hidden (128 default, 512 = the reference's). Reports ms and the
effective HBM rate (bytes the kernel must move: fwd x (+res) + y + mean/rstd, bwd dy + x +
dx + mean/rstd) for forward, forward+residual and backward.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="655320,1038240,1618752,3114720")
    ap.add_argument("--hidden", default="128,512")
    a = ap.parse_args()
    from dgraph_amd import _native

    assert _native.load(), "native library missing"
    ops = _native.ops()
    dev = torch.device("cuda")
    for F in [int(v) for v in a.hidden.split(",")]:
        for N in [int(v) for v in a.rows.split(",")]:
            x = torch.randn(N, F, device=dev).bfloat16()
            r = torch.randn(N, F, device=dev).bfloat16()
            dy = torch.randn(N, F, device=dev).bfloat16()
            g = torch.rand(F, device=dev) + 0.5
            b = torch.randn(F, device=dev)
            y, mean, rstd = ops.layer_norm_fwd(x, g, b, None, 1e-5)
            t_f = timeit(lambda: ops.layer_norm_fwd(x, g, b, None, 1e-5))
            t_fr = timeit(lambda: ops.layer_norm_fwd(x, g, b, r, 1e-5))
            t_b = timeit(lambda: ops.layer_norm_bwd(dy, x, mean, rstd, g))
            e = 2 * N * F
            rec = dict(N=N, F=F, fwd_ms=round(t_f, 4), fwd_res_ms=round(t_fr, 4),
                       bwd_ms=round(t_b, 4),
                       fwd_TBs=round((2 * e + 8 * N) / t_f / 1e9, 2),
                       fwd_res_TBs=round((3 * e + 8 * N) / t_fr / 1e9, 2),
                       bwd_TBs=round((3 * e + 8 * N) / t_b / 1e9, 2))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
