"""API-compatibility module: reference path ``DGraph.torch_nvshmem_p2p (native extension)`` re-exported from ``dgraph_amd.comm.symheap``
(dgraph_amd is the implementation; this tree only preserves DGraph import paths)."""
from dgraph_amd.comm.symheap import NVSHMEMP2P  # noqa: F401
