"""API-compatibility module: reference path ``DGraph/distributed/mpi/MPIBackendEngine.py`` re-exported from ``dgraph_amd.comm.mpi_engine``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.comm.mpi_engine import MPIBackendEngine  # noqa: F401
