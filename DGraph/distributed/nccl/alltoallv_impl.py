"""API-compatibility module: reference path ``DGraph/distributed/nccl/alltoallv_impl.py`` re-exported from ``dgraph_amd.comm.alltoallv``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.comm.alltoallv import (AllToAllV, _nccl_alltoallv_with_dict,  # noqa: F401
                                       offsets_to_splits, torch_alltoallv_with_comm_map)
