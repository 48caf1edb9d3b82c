"""API-compatibility module: reference path ``DGraph/distributed/nccl/__init__.py`` re-exported from ``dgraph_amd.comm / dgraph_amd.plan``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.comm.nccl_engine import TIMINGS, NCCLBackendEngine  # noqa: F401
from dgraph_amd.plan.nccl_plan import (  # noqa: F401
    COO_to_NCCLCommPlan, COO_to_NCCLEdgeConditionedCommPlan, NCCLEdgeConditionedGraphCommPlan,
    NCCLGraphCommPlan)
