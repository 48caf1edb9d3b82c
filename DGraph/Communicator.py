"""API-compatibility module: reference path ``DGraph/Communicator.py`` re-exported from ``dgraph_amd.comm.communicator``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.comm.communicator import SUPPORTED_BACKENDS, Communicator  # noqa: F401
from dgraph_amd.comm.base import CommunicatorBase  # noqa: F401
