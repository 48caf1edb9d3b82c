#!/usr/bin/env python3
"""Fused one-kernel hidden layers vs the chunked path on the full headline graph: one
forward+backward from identical weights, compare sampled hidden rows, loss and the role
synchronisation error flag."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import bench
    import dgraph_amd.models.sage_fused as sf
    from dgraph_amd import Communicator

    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    args = bench.parse.__wrapped__() if hasattr(bench.parse, "__wrapped__") else None
    sys.argv = [sys.argv[0], "--scale", str(a.scale)]
    args = bench.parse()
    comm = Communicator.init_process_group("nccl")
    dev = torch.device("cuda", 0)
    sf.FUSED_FWD = True
    job = bench.Job(args, comm, dev, args.global_frac, torch.float32)
    ex = job.fused
    state = {k: v.clone() for k, v in job.model.state_dict().items()}
    L = ex.L
    rows = torch.randint(0, L, (1 << 14,), device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    out = {}
    for mode in ("chunked", "fused"):
        job.model.load_state_dict(state)
        ring = ex.fwd_ring
        if mode == "chunked":
            ex.fwd_ring = None
        loss = ex.step()
        ex.fwd_ring = ring
        torch.cuda.synchronize()
        out[mode] = (float(loss), ex.h[0][rows].clone(), ex.h[1][rows].clone() if False else None)
        print(mode, "loss", float(loss), "err", int(ex.fwd_err.item()), flush=True)
        # h[1] is overwritten by the backward (dZ/u live in it); compare h[0] (layer-0 output)
    l0, h0a, _ = out["chunked"]
    l1, h0b, _ = out["fused"]
    d = (h0a - h0b).abs()
    print("h1 rows: equal", torch.equal(h0a, h0b), "max abs diff", float(d.max()),
          "n diff", int((d > 0).sum()), "loss diff", l1 - l0, flush=True)


if __name__ == "__main__":
    main()
