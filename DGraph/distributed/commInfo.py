"""API-compatibility module: reference path ``DGraph/distributed/commInfo.py`` re-exported from ``dgraph_amd.plan.pattern``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.plan.pattern import (  # noqa: F401
    CommunicationPattern, build_communication_pattern, compute_boundary_vertices,
    compute_comm_map, compute_halo_vertices, compute_local_edge_list, compute_local_vertices,
    compute_recv_offsets)
