"""API-compatibility module: reference path ``DGraph/distributed/nccl/_NCCLCommPlan.py`` re-exported from ``dgraph_amd.plan.nccl_plan``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.plan.nccl_plan import (  # noqa: F401
    COO_to_NCCLCommPlan, COO_to_NCCLEdgeConditionedCommPlan, NCCLEdgeConditionedGraphCommPlan,
    NCCLGraphCommPlan, compute_edge_slices, fast_2D_unique)
