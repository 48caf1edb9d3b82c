"""API-compatibility module: reference path ``DGraph/distributed/haloExchange.py`` re-exported from ``dgraph_amd.parallel.halo``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.parallel.halo import DGraphMessagePassing, HaloExchange, HaloExchangeImpl  # noqa: F401
