"""API-compatibility module: reference path ``DGraph/distributed/nccl/NCCLBackendEngine.py`` re-exported from ``dgraph_amd.comm.nccl_engine``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.comm.nccl_engine import TIMINGS, NCCLBackendEngine  # noqa: F401
