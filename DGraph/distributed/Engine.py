"""API-compatibility module: reference path ``DGraph/distributed/Engine.py`` re-exported from ``dgraph_amd.comm.base``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.comm.base import BackendEngine  # noqa: F401
