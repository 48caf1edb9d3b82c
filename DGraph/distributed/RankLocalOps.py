"""API-compatibility module: reference path ``DGraph/distributed/RankLocalOps.py`` re-exported from ``dgraph_amd.parallel.rank_local``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.parallel.rank_local import *  # noqa: F401,F403
from dgraph_amd.ops.local import (  # noqa: F401
    local_masked_gather, local_masked_scatter, local_masked_scatter_add_gather,
    local_masked_scatter_gather)
_LOCAL_OPT_KERNELS_AVAILABLE = True
