"""API-compatibility module: reference path ``DGraph/__init__.py`` re-exported from ``dgraph_amd``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd import Communicator, CommunicatorBase, __version__  # noqa: F401
