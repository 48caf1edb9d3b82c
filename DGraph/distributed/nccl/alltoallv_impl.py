"""API-compatibility module: reference path ``DGraph/distributed/nccl/alltoallv_impl.py`` re-exported from ``dgraph_amd.comm.alltoallv``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.comm.alltoallv import AllToAllV, offsets_to_splits  # noqa: F401
