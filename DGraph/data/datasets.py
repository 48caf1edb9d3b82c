"""API-compatibility module: reference path ``DGraph/data/datasets.py`` re-exported from ``dgraph_amd.data.ogbn``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.data.ogbn import DistributedOGBWrapper  # noqa: F401
