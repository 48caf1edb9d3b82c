"""API-compatibility module: reference path ``DGraph/checks.py`` re-exported from ``dgraph_amd.utils``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.utils import check_dist_initialized, check_nccl_availability  # noqa: F401
