"""API-compatibility module: reference path ``DGraph/distributed/nvshmem/NVSHMEMBackendEngine.py`` re-exported from ``dgraph_amd.comm.shmem_engine``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.comm.shmem_engine import NVSHMEMBackendEngine, ROCSHMEMBackendEngine  # noqa: F401
