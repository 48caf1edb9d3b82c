"""API-compatibility module: reference path ``DGraph/utils/data_splitting.py`` re-exported from ``dgraph_amd.utils.data_splitting``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.utils.data_splitting import largest_split  # noqa: F401
