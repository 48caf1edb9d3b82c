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
from .__version__ import __version__
from .comm.base import BackendEngine, CommunicatorBase
from .comm.communicator import SUPPORTED_BACKENDS, Communicator

__all__ = ["Communicator", "CommunicatorBase", "BackendEngine", "SUPPORTED_BACKENDS",
           "__version__"]
