"""API-compatibility module: reference path ``DGraph/distributed/nccl/_nccl_cache.py`` re-exported from ``dgraph_amd.plan.legacy_cache``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.plan.legacy_cache import (  # noqa: F401
    NCCLGatherCache, NCCLGatherCacheGenerator, NCCLScatterCache, NCCLScatterCacheGenerator,
    load_cache, save_cache)
