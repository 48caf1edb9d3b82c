"""API-compatibility module: reference path ``DGraph/data/preprocess.py`` re-exported from ``dgraph_amd.data.preprocess``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.data.preprocess import (  # noqa: F401
    edge_renumbering, node_renumbering, process_homogenous_data)
