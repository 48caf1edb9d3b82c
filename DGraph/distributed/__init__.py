"""API-compatibility module: reference path ``DGraph/distributed/__init__.py`` re-exported from ``dgraph_amd.parallel / dgraph_amd.plan``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.parallel.halo import DGraphMessagePassing, HaloExchange  # noqa: F401
from dgraph_amd.plan.pattern import CommunicationPattern, build_communication_pattern  # noqa: F401
