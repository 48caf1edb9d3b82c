"""API-compatibility module: reference path ``DGraph/utils/__init__.py`` re-exported from ``dgraph_amd.utils``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.utils import try_barrier  # noqa: F401
from dgraph_amd.utils.data_splitting import largest_split, split_per_rank  # noqa: F401
