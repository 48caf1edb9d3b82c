"""API-compatibility module: reference path ``DGraph/data/graph.py`` re-exported from ``dgraph_amd.data.graph``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.data.graph import DistributedGraph, get_round_robin_node_rank_map  # noqa: F401
