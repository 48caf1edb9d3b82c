"""API-compatibility module: reference path ``DGraph/CommunicatorBase.py`` re-exported from ``dgraph_amd.comm.base``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.comm.base import CommunicatorBase  # noqa: F401
