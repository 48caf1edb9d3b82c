"""API-compatibility module: reference path ``DGraph/distributed/nccl/_torch_func_impl.py`` re-exported from ``dgraph_amd.parallel``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.parallel.index_ops import GatherFunction, ScatterFunction  # noqa: F401
from dgraph_amd.parallel.plan_ops import CommPlan_GatherFunction, CommPlan_ScatterFunction  # noqa: F401
