#!/usr/bin/env python3
"""Micro-benchmark of the CSR SpMM aggregation kernel variants on a synthetic graph.

Interleaved A/B rounds in one process (cdna_hip_programming.md §5.4 rule 24); reports
median ms and effective bytes/s (gathered neighbour rows + indices + output rows).
Example: python benchmarks/bench_spmm.py --shape ogbn-papers100M --feats 128,172,256
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="ogbn-products")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--feats", default="128,172,256")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--global-frac", type=float, default=0.05)
    ap.add_argument("--window", type=int, default=1 << 14)
    ap.add_argument("--variants", default="2:2:128,4:0:128,4:2:64",
                    help="comma list of variant:row_map:pass_cols[:hub_cap] (hub_cap > 0: "
                         "hub-row split at that degree)")
    ap.add_argument("--slices", default="1")
    ap.add_argument("--powerlaw", type=float, default=0.0,
                    help="> 0: instead of the shaped generator, a power-law in-degree graph: "
                         "row = floor(V u^a) for u ~ U(0,1) (a = 6: the top row holds ~5%% "
                         "of all entries), uniform columns, E_msg entries")
    ap.add_argument("--mean", default="row", choices=["row", "col"],
                    help="mean as a row scale (forward) or a column scale (transposed)")
    a = ap.parse_args()
    from dgraph_amd import _native
    from dgraph_amd.data.synthetic import SHAPES, build_partition
    from dgraph_amd.ops import kernels as K

    ops = _native.ops()
    dev = torch.device("cuda", 0)
    shape = SHAPES[a.shape] if a.scale == 1.0 else SHAPES[a.shape].scaled(a.scale)
    if a.powerlaw > 0:
        from dgraph_amd.ops.csr import CSR

        V, E = shape.num_nodes, 2 * shape.num_directed_edges
        gen = torch.Generator(device=dev).manual_seed(0)
        rows = (torch.rand(E, generator=gen, device=dev) ** a.powerlaw * V).long()
        rows.clamp_(max=V - 1)
        rows, _ = torch.sort(rows)
        cols = torch.randint(0, V, (E,), generator=gen, device=dev, dtype=torch.int32)
        csr = CSR.from_coo(rows, cols, V, V, keep_perm=False)
        del rows, cols
        p = {"csr": csr, "L": V}
    else:
        p = build_partition(shape, 0, 1, dev, global_frac=a.global_frac, window=a.window)
    csr = p["csr"]
    deg = csr.degree()
    q = torch.quantile(deg[:: max(1, deg.numel() // (1 << 22))].float(),
                       torch.tensor([0.5, 0.99, 0.9999], device=dev))
    print(f"[spmm] rows={csr.num_rows} nnz={csr.nnz} degree median/p99/p99.99/max = "
          f"{q.tolist()} / {int(deg.max())}; rows > 256: {int((deg > 256).sum())}, "
          f"> 4096: {int((deg > 4096).sum())}", flush=True)
    inv = csr.inv_degree()
    sc = {"row_scale": inv} if a.mean == "row" else {"col_scale": inv}
    variants = [tuple(int(v) for v in s.split(":")) for s in a.variants.split(",")]
    res = {}
    for F in [int(f) for f in a.feats.split(",")]:
        x = torch.randn(p["L"], F, device=dev, dtype=torch.bfloat16)
        out = torch.empty_like(x)
        times = {v: [] for v in variants}
        ref = None
        for r in range(a.rounds + 1):
            for v in variants:
                ops.set_spmm_config(*v[:3])
                sp = csr.hub_split(v[3]) if len(v) > 3 else None
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                s.record()
                K.spmm(csr.rowptr, csr.col, x, out, split=sp, **sc)
                e.record()
                torch.cuda.synchronize()
                if r > 0:
                    times[v].append(s.elapsed_time(e))
                if ref is None:
                    ref = out.clone()
                else:  # variants sum in different orders: compare to rounding
                    rows = torch.arange(0, out.shape[0], 997, device=out.device)
                    err = (out[rows].float() - ref[rows].float()).abs().max().item()
                    assert err < 5e-2, f"variant {v} differs by {err}"
        nbytes = csr.nnz * (F * 2 + csr.col.element_size()) + p["L"] * F * 2
        # feature-sliced execution (narrower gathered rows -> smaller per-XCD working set)
        for s, v in [(int(sv), v) for sv in a.slices.split(",") for v in variants
                     if int(sv) > 1 and F % int(sv) == 0]:
            ops.set_spmm_config(*v[:3])
            ts = []
            w = F // s
            for r in range(a.rounds + 1):
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                st.record()
                for j in range(s):
                    K.spmm(csr.rowptr, csr.col, x[:, j * w:(j + 1) * w],
                           out[:, j * w:(j + 1) * w], **sc)
                en.record()
                torch.cuda.synchronize()
                if r > 0:
                    ts.append(st.elapsed_time(en))
            ms = statistics.median(ts)
            res[f"F{F}_slices{s}_v{v[0]}_xcd{v[1]}"] = {"ms": round(ms, 3),
                                                         "TBps": round(nbytes / ms / 1e9, 3)}
            print(f"F={F:4d} slices={s} variant={v[0]} xcd={v[1]}: {ms:8.2f} ms  {nbytes / ms / 1e9:6.2f} TB/s effective",
                  flush=True)
        for v in variants:
            ms = statistics.median(times[v])
            res[f"F{F}_" + "_".join(str(t) for t in v)] = {"ms": round(ms, 3),
                                                          "TBps": round(nbytes / ms / 1e9, 3)}
            print(f"F={F:4d} variant={v} window={a.window}: {ms:8.2f} ms  "
                  f"{nbytes / ms / 1e9:6.2f} TB/s effective", flush=True)
        del x, out, ref
    ops.set_spmm_config(-1, -1)
    print(json.dumps({"shape": shape.name, "nnz": csr.nnz, "rows": p["L"], "results": res}))


if __name__ == "__main__":
    main()
