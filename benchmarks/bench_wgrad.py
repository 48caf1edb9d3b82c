"""Weight-gradient (x^T g, L ~ 1e8 rows) variants on one GPU: chunk sizes of the batched
split-K formulation vs a plain GEMM. Prints one line per variant (ms per call)."""
import argparse
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgraph_amd.ops.dense import mm_f32, wgrad  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=111_059_956)
    ap.add_argument("--shapes", default="256x256,128x256,256x128,256x172")
    a = ap.parse_args()
    dev = torch.device("cuda")
    L = a.rows
    for sh in a.shapes.split(","):
        K, N = (int(v) for v in sh.split("x"))
        x = torch.randn(L, K, device=dev, dtype=torch.bfloat16)
        g = torch.randn(L, N, device=dev, dtype=torch.bfloat16)
        gb = (L * (K + N) * 2) / 1e9
        res = {}
        res["default"] = timeit(lambda: wgrad(x, g))
        for rpc in (1 << 12, 1 << 13, 1 << 14, 1 << 15, 1 << 18):
            res[f"bmm rpc={rpc}"] = timeit(lambda: wgrad(x, g, rpc))
        res["mm"] = timeit(lambda: mm_f32(x.t(), g))
        for k, v in res.items():
            print(f"K={K} N={N} {k:24s} {v:8.2f} ms  {gb / v:6.2f} TB/s-equiv", flush=True)
        del x, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
