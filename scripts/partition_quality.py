"""Partition quality at the papers100M scale.

Generates the synthetic papers100M-shaped graph that bench.py trains on (all 1.6e9 directed
pairs, on one GPU), then reports for W in {2, 4, 8}: the edge cut, the total and max
pairwise halo (rows rank q must receive from rank p; the MAX pair bounds an all-to-all-v
over point-to-point xGMI), per-rank max halo and the size imbalance, for

  contiguous      the id-block partition bench.py uses
  lp(contiguous)  balanced label propagation refining it
  random          seeded uniform (W=8 only)
  lp(random)      label propagation from the random start (W=8 only: shows the
                  partitioner recovering locality at this scale)

for both localities (--global-fracs, default 0.05 and 1.0). One JSON line per result.
"""
import argparse
import json
import time

import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from dgraph_amd.data.partition import (contiguous_partition, label_propagation_partition,
                                       partition_stats, random_partition)
from dgraph_amd.data.synthetic import _CHUNK, SHAPES, _chunk_edges


def gen_edges(shape, gf, window, dev):
    E = shape.num_directed_edges
    ei = torch.empty(2, E, dtype=torch.int64, device=dev)
    for k in range(0, (E + _CHUNK - 1) // _CHUNK):
        n = min(_CHUNK, E - k * _CHUNK)
        s, d = _chunk_edges(shape, k, n, 0, gf, window, dev)
        ei[0, k * _CHUNK:k * _CHUNK + n] = s
        ei[1, k * _CHUNK:k * _CHUNK + n] = d
    return ei


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="ogbn-papers100M")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--global-fracs", default="0.05,1.0")
    ap.add_argument("--window", type=int, default=1 << 14)
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--imbalance", type=float, default=0.05)
    ap.add_argument("--out", default="gpurun_out/partition_quality.jsonl")
    a = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    shape = SHAPES[a.shape]
    if a.scale != 1.0:
        shape = shape.scaled(a.scale)
    V = shape.num_nodes
    out = open(a.out, "w")

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        out.write(line + "\n")
        out.flush()

    for gf in [float(x) for x in a.global_fracs.split(",")]:
        t = time.time()
        ei = gen_edges(shape, gf, a.window, dev)
        print(f"[pq] global_frac={gf}: {ei.shape[1]} directed pairs in {time.time() - t:.1f}s",
              flush=True)
        for W in [int(x) for x in a.worlds.split(",")]:
            cases = [("contiguous", lambda: contiguous_partition(V, W, dev)),
                     ("lp(contiguous)", lambda: label_propagation_partition(
                         ei, V, W, rounds=a.rounds, imbalance=a.imbalance))]
            if W == 8:
                cases += [("random", lambda: random_partition(V, W, seed=0, device=dev)),
                          ("lp(random)", lambda: label_propagation_partition(
                              ei, V, W, rounds=2 * a.rounds, imbalance=a.imbalance,
                              init=random_partition(V, W, seed=0, device=dev)))]
            for name, fn in cases:
                t = time.time()
                part = fn()
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                tp = time.time() - t
                t = time.time()
                st = partition_stats(ei, part, W, symmetric=True)
                pm = st.pop("pair_matrix")
                emit(dict(shape=a.shape, scale=a.scale, V=V, E_directed=int(ei.shape[1]),
                          global_frac=gf, window=a.window, world=W, partition=name,
                          partition_s=round(tp, 2), stats_s=round(time.time() - t, 2),
                          **st, halo_bytes_max_pair_f128_bf16=st["halo_rows_max_pair"] * 256,
                          pair_matrix=pm.tolist()))
                del part
        del ei
        if dev.type == "cuda":
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
