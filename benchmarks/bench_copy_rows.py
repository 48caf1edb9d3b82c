"""Row-gather rate of ``K.copy_rows`` at the streamed-halo pack shape.

The structureless W=8 rank packs ~10^8 send rows per 64-column block out of a [L, 256]
fp32 activation (rows sorted by source, scattered destinations: ``FusedSAGE._pack``).
Prints one JSON line per configuration: ms per call and the GB/s of bytes read + written.

    python benchmarks/bench_copy_rows.py [--rows 14000000] [--send 60000000]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=14_000_000)
    ap.add_argument("--send", type=int, default=60_000_000)
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from dgraph_amd import _native
    from dgraph_amd.ops import kernels as K

    assert _native.load(), "native library missing"
    dev = torch.device("cuda", 0)
    x = torch.randn(a.rows, a.width, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    src = torch.randint(0, a.rows, (a.send,), device=dev, generator=g)
    order = torch.argsort(src, stable=True)
    cases = {
        "source_sorted": (src[order].int().contiguous(), order.int().contiguous()),
        "destination_order": (src.int().contiguous(), None),
    }
    for cw in (64, 256):
        out = torch.empty(a.send, cw, device=dev)
        xs = x[:, :cw]
        for name, (si, di) in cases.items():
            K.copy_rows(xs, src_idx=si, dst_idx=di, out=out)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                K.copy_rows(xs, src_idx=si, dst_idx=di, out=out)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.iters
            byts = 2 * a.send * cw * 4
            print(json.dumps({"bench": "copy_rows", "order": name, "rows": a.send,
                              "columns": cw, "ld": a.width, "ms": round(ms, 3),
                              "GBps_read_plus_written": round(byts / ms / 1e6, 1)}),
                  flush=True)
        del out


if __name__ == "__main__":
    main()
