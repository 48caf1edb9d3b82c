"""API-compatibility module: reference path ``DGraph/distributed/nccl/_indices_utils.py`` re-exported from ``dgraph_amd.plan.legacy_cache``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.plan.legacy_cache import (  # noqa: F401
    _generate_local_rank_mapping, _get_local_send_placement, _get_recv_comm_vector,
    _get_send_comm_vector, _get_send_recv_comm_vectors)
