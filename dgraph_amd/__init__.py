"""dgraph_amd — distributed full-graph GNN training, native to AMD Instinct MI355X (gfx950).

A from-scratch framework with the capabilities and public API of LBANN/DGraph:
vertex-partitioned graphs, autograd-aware halo exchange and distributed vertex<->edge
gather / scatter-sum, over RCCL (xGMI) all-to-all-v, a host-capable "mpi" engine and a
one-sided symmetric-heap engine; local message passing runs in hand-written CDNA4 HIP
kernels (``csrc/``), loaded as ``torch.ops.dgraph_amd``.

Layout:
    dgraph_amd.comm      Communicator + backend engines + all-to-all-v executor
    dgraph_amd.plan      CommunicationPattern (G3), NCCLGraphCommPlan (G2), caches (G1)
    dgraph_amd.ops       native kernels, CSR, autograd sparse primitives
    dgraph_amd.parallel  halo exchange, plan ops, index ops, DistGraph, sync-BN, DP
    dgraph_amd.models    GraphSAGE, GCN (DGraph OGB), GAT/RGAT, R-GCN, GraphCast
    dgraph_amd.data      DistributedGraph, preprocessing, partitioners, synthetic graphs
    dgraph_amd.utils     TimingReport, metrics, config, checkpointing
"""
import os as _os

# (ProcessGroupNCCL keeps an asynchronous collective's tensors alive until its work.wait()
# instead of record_stream-ing them — the default of this torch; the library's own
# transports do the same, comm/alltoallv.py _EventWork.)


def _hw_queues() -> None:
    """At least 8 hardware queues per process (HIP's default, and the GPU boxes' exported
    value, is 4): with 4, torch's pool streams share queues with the compute stream, and a
    comm stream on the compute stream's queue runs in order with it — no overlap
    (PERFORMANCE.md, round 5). Only before the HIP runtime starts; DGRAPH_HW_QUEUES sets
    the value explicitly."""
    import sys

    t = sys.modules.get("torch")
    if t is not None and t.cuda.is_initialized():
        return
    want = _os.environ.get("DGRAPH_HW_QUEUES")
    cur = _os.environ.get("GPU_MAX_HW_QUEUES", "")
    if want:
        _os.environ["GPU_MAX_HW_QUEUES"] = want
    elif not cur.isdigit() or int(cur) < 8:
        _os.environ["GPU_MAX_HW_QUEUES"] = "8"


_hw_queues()

from .__version__ import __version__  # noqa: E402
from .comm.base import BackendEngine, CommunicatorBase  # noqa: E402
from .comm.communicator import SUPPORTED_BACKENDS, Communicator  # noqa: E402

__all__ = ["Communicator", "CommunicatorBase", "BackendEngine", "SUPPORTED_BACKENDS",
           "__version__"]
