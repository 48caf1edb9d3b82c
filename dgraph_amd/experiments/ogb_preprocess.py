"""OGB graph preprocessing: networkx pickles, partitioning, renumbering, placement files.

Counterpart of experiments/OGB/preprocess.py:15-131. The reference needs ``metis`` (and
``fire``); here the partitioner is chosen by availability:

  ``metis``  the ``metis`` Python binding (``networkx_to_metis`` + ``part_graph``), as in
             the reference, when importable;
  ``pymetis`` the ``pymetis`` binding (CSR adjacency), when importable;
  ``lp``     the library's balanced label propagation (:mod:`dgraph_amd.data.partition`,
             vectorised torch, on the GPU when one is present; the 1.6e9-edge papers100M
             graph partitions in ~4 s on one MI355X, profiles/partition_quality_papers100M.txt);

``--method auto`` takes the first available. Neither METIS binding is installed in this
image, so ``auto`` resolves to ``lp`` here (METIS parity unpinned; the wiring is tested
with a stand-in module).

Outputs (``--out_dir``):

* ``{dname}_directed={bool}.pkl`` — the networkx graph, the reference's layout
  (``save_networkx_graph``; arxiv is saved directed with both edge directions added, the
  others undirected). These are pickles: :func:`load_networkx_graph` unpickles, so load
  only files this tool wrote.
* ``{dname}_placement_W{W}.pt`` — per-vertex owner rank (int64 tensor, ``torch.save``), the
  ``--node_rank_placement_file`` that :mod:`dgraph_amd.experiments.ogb_gcn` and
  ``examples/ogb/generate_cache.py`` load with ``weights_only=True``;
* ``{dname}_placement_W{W}.json`` — edge cut, total / max-pairwise halo rows, imbalance.

Renumbering uses :mod:`dgraph_amd.data.preprocess` (old->new through the inverse
permutation; the reference relabelled with new->old).

    python -m dgraph_amd.experiments.ogb_preprocess --dset_name ogbn-arxiv --num_ranks 8
"""
from __future__ import annotations

import argparse
import json
import os
import pickle
from typing import Optional, Tuple

import numpy as np
import torch

from ..data.partition import (contiguous_partition, label_propagation_partition,
                              partition_stats)
from ..data.preprocess import add_opposite_edges, edge_renumbering, node_renumbering

__all__ = ["partition_graph", "partition_directed_graph", "save_networkx_graph",
           "load_networkx_graph", "add_opposite_edges", "available_methods", "main"]


def available_methods():
    out = []
    for m in ("metis", "pymetis"):
        try:
            __import__(m)
            out.append(m)
        except ImportError:
            pass
    return out + ["lp"]


def _coo_tensor(coo_list) -> torch.Tensor:
    """[E, 2] (the reference's coo_list) or [2, E] -> int64 [2, E]."""
    t = torch.as_tensor(np.asarray(coo_list)).long()
    if t.dim() != 2:
        raise ValueError("edge list must be 2-D")
    return t.t().contiguous() if t.shape[1] == 2 and t.shape[0] != 2 else t


def _placement(ei: torch.Tensor, num_nodes: int, num_parts: int, method: str,
               directed: bool, lp_rounds: int = 20, seed: int = 0) -> torch.Tensor:
    if method == "auto":
        method = available_methods()[0]
    if method == "metis":
        import metis  # type: ignore
        import networkx as nx

        G = nx.DiGraph() if directed else nx.Graph()
        G.add_nodes_from(range(num_nodes))
        G.add_edges_from(ei.t().tolist())
        _, parts = metis.part_graph(metis.networkx_to_metis(G), nparts=num_parts)
        return torch.as_tensor(np.asarray(parts), dtype=torch.long)
    if method == "pymetis":
        import pymetis  # type: ignore

        sym = add_opposite_edges(ei)
        sym = sym[:, sym[0] != sym[1]]
        sym = torch.unique(sym, dim=1)
        deg = torch.bincount(sym[0], minlength=num_nodes)
        xadj = torch.zeros(num_nodes + 1, dtype=torch.long)
        xadj[1:] = torch.cumsum(deg, 0)
        _, parts = pymetis.part_graph(num_parts, xadj=xadj.numpy(), adjncy=sym[1].numpy())
        return torch.as_tensor(np.asarray(parts), dtype=torch.long)
    if method in ("lp", "label_propagation"):
        dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        part = label_propagation_partition(ei.to(dev), num_nodes, num_parts, rounds=lp_rounds,
                                           init=contiguous_partition(num_nodes, num_parts, dev),
                                           seed=seed)
        return part.cpu()
    raise ValueError(f"unknown partition method {method!r} (have {available_methods()})")


def partition_graph(coo_list, num_ranks: int, num_nodes: Optional[int] = None,
                    method: str = "auto", directed: bool = False
                    ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Partition, then renumber so every rank owns a contiguous id block.

    Returns ``(new_to_old, renumbered_edges[2, E], placement)`` where ``placement[v]`` is
    the owner of ORIGINAL vertex ``v`` (what the placement file stores)."""
    ei = _coo_tensor(coo_list)
    n = int(num_nodes) if num_nodes is not None else int(ei.max()) + 1
    placement = _placement(ei, n, num_ranks, method, directed)
    new_to_old, ranks_of_new = node_renumbering(placement)
    edges, _, _, _ = edge_renumbering(ei, new_to_old, ranks_of_new)
    return new_to_old, edges, placement


def partition_directed_graph(coo_list, num_nodes: int, num_parts: int, method: str = "auto"):
    """The directed variant (reference :32-47, minus its ``breakpoint()``)."""
    return partition_graph(coo_list, num_parts, num_nodes, method, directed=True)


def save_networkx_graph(coo_list, num_nodes: int, dname: str, directed: bool = False,
                        out_dir: str = ".") -> str:
    """``{out_dir}/{dname}_directed={directed}.pkl``: all vertices plus the edges; a
    directed graph also gets every reverse edge (reference :83-99)."""
    import networkx as nx

    ei = _coo_tensor(coo_list)
    G = nx.DiGraph() if directed else nx.Graph()
    G.add_nodes_from(range(int(num_nodes)))
    pairs = ei.t().tolist()
    G.add_edges_from(pairs)
    if directed:
        G.add_edges_from((d, s) for s, d in pairs)
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, f"{dname}_directed={directed}.pkl")
    with open(path, "wb") as f:
        pickle.dump(G, f)
    return path


def load_networkx_graph(dname: str):
    """Unpickle ``{dname}.pkl`` (``dname`` includes the ``_directed=...`` suffix, as in the
    reference). Pickles execute code on load: only load files this tool wrote."""
    with open(f"{dname}.pkl", "rb") as f:
        return pickle.load(f)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--dset_name", default="ogbn-arxiv")
    ap.add_argument("--num_ranks", type=int, default=0,
                    help="also partition into this many ranks and write the placement file")
    ap.add_argument("--method", default="auto", help="auto | metis | pymetis | lp")
    ap.add_argument("--out_dir", default=".")
    ap.add_argument("--root_dir", default="data")
    ap.add_argument("--scale", type=float, default=1.0, help="synthetic-graph scale (no ogb)")
    ap.add_argument("--no_networkx", action="store_true", help="skip the networkx pickle")
    a = ap.parse_args(argv)
    from ..data.ogbn import _load_ogb, _synthetic_ogb

    name = a.dset_name if a.dset_name.startswith("ogbn-") else f"ogbn-{a.dset_name}"
    try:
        graph, _, _ = _load_ogb(name, a.root_dir)
        source = "ogb"
    except Exception:  # noqa: BLE001 - no ogb / no files: synthetic graph of that shape
        graph, _, _ = _synthetic_ogb(name, scale=a.scale)
        source = f"synthetic@{a.scale}"
    ei = torch.as_tensor(np.asarray(graph["edge_index"])).long()
    V = int(graph["num_nodes"])
    directed = name == "ogbn-arxiv"
    os.makedirs(a.out_dir, exist_ok=True)
    if not a.no_networkx:
        print("wrote", save_networkx_graph(ei, V, name, directed=directed, out_dir=a.out_dir))
    if a.num_ranks > 0:
        method = available_methods()[0] if a.method == "auto" else a.method
        _, _, placement = partition_graph(ei, a.num_ranks, V, method, directed)
        base = os.path.join(a.out_dir, f"{name}_placement_W{a.num_ranks}")
        torch.save(placement, base + ".pt")
        st = partition_stats(ei, placement, a.num_ranks, symmetric=True)
        st["pair_matrix"] = st["pair_matrix"].tolist()
        st.update(dataset=name, source=source, method=method, num_nodes=V,
                  num_edges=int(ei.shape[1]), world_size=a.num_ranks)
        with open(base + ".json", "w") as f:
            json.dump(st, f, indent=1)
        print("wrote", base + ".pt", {k: st[k] for k in ("method", "edge_cut_frac",
                                                          "halo_rows_max_pair", "imbalance")})
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
