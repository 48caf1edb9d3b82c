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
# (ProcessGroupNCCL keeps an asynchronous collective's tensors alive until its work.wait()
# instead of record_stream-ing them — the default of this torch; the library's own
# transports do the same, comm/alltoallv.py _EventWork.)
#
# GPU_MAX_HW_QUEUES is left as the operator set it (the boxes export HIP's default, 4): the
# halo exchange runs on a HIGH-priority stream (comm/alltoallv.py _side_stream, RCCL's
# stream in comm/groups.py), which the runtime places on a queue of its own whatever the
# queue budget (scripts/debug/queue_probe.py), so overlap does not depend on raising it.

from .__version__ import __version__  # noqa: E402
from .comm.base import BackendEngine, CommunicatorBase  # noqa: E402
from .comm.communicator import SUPPORTED_BACKENDS, Communicator  # noqa: E402

__all__ = ["Communicator", "CommunicatorBase", "BackendEngine", "SUPPORTED_BACKENDS",
           "__version__"]
