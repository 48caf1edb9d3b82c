#!/usr/bin/env python3
"""Per-parameter gradient error of the fused executor at W=1 on the GPU kernels against the
same executor on the CPU (fp64 references), at hidden 256 / 384 / 512."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402


def grads(dev, hidden, part, x0, y0, split0, shape):
    from dgraph_amd.data.synthetic import SPLIT_TEST, SPLIT_TRAIN, SPLIT_VALID
    from dgraph_amd.models.sage import GraphSAGE
    from dgraph_amd.models.sage_fused import FusedSAGE
    from dgraph_amd.parallel.dist_graph import DistGraph

    x, y, split = x0.to(dev), y0.to(dev), split0.to(dev)
    csr = part["csr"].to(dev)
    tr = torch.nonzero(split == SPLIT_TRAIN).reshape(-1)
    ev = torch.nonzero((split == SPLIT_VALID) | (split == SPLIT_TEST)).reshape(-1)
    torch.manual_seed(0)
    model = GraphSAGE(shape.num_features, hidden, shape.num_classes, 3).to(dev)
    g = DistGraph(csr, part["L"], 0, symmetric=True)
    ex = FusedSAGE(model, g, x, tr, y[tr], ev, y[ev], split[ev] == SPLIT_VALID, tr.numel(),
                   chunk_rows=int(os.environ.get("CHUNK", "2048")))
    loss = ex.step()
    return float(loss), [p.grad.detach().double().cpu() for p in model.parameters()]


def main():
    from dgraph_amd.data.synthetic import SHAPES, build_partition, contiguous_offsets, node_data

    shape = SHAPES["ogbn-papers100M"].scaled(2e-4)
    part = build_partition(shape, 0, 1, "cpu", global_frac=0.05, window=256)
    part["csr"].num_cols = part["L"]
    x0, y0, split0 = node_data(shape, 0, contiguous_offsets(shape.num_nodes, 1), "cpu",
                               dtype=torch.float32, return_split=True)
    names = [f"l{i}.{n}" for i in range(3) for n in ("w_self", "w_neigh", "bias")]
    for h in [int(v) for v in sys.argv[1:]] or [256, 512]:
        lc, gc = grads("cpu", h, part, x0, y0, split0, shape)
        lg, gg = grads("cuda", h, part, x0, y0, split0, shape)
        print(f"hidden {h}: loss gpu {lg:.8f} cpu {lc:.8f}", flush=True)
        for n, a, b in zip(names, gg, gc):
            rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
            print(f"  {n:12s} rel {rel:.3e}", flush=True)


if __name__ == "__main__":
    main()
