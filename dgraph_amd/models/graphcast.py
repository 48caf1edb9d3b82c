"""GraphCast encoder-processor-decoder (experiments/GraphCast/{layers,model}.py).

Layer structure and parameter names follow the reference (``MeshGraphMLP._model`` =
Linear, SiLU, [Linear, SiLU]*, Linear, LayerNorm), so state dicts are interchangeable.
The MI355X formulation of the hot blocks:

* ``MeshEdgeBlock``: ``e' = MLP([x_src[s] || x_dst[d] || e]) + e``. The first Linear is
  distributed over the concatenation: vertex-level GEMMs ``P = x_src W_s^T``,
  ``Q = x_dst W_d^T`` plus the edge GEMM ``Y = e W_e^T + b``, fused with the gathers and the
  SiLU in ONE edge kernel (``gather_add_act``; the pre-activation is recomputed in backward,
  never stored). No ``E x 3F`` concatenation is ever built.
* ``MeshNodeBlock``: ``x' = MLP([x || sum_{e -> x} e]) + x`` with the edge sum a
  destination-sorted CSR segment reduction (deterministic, no atomics) and the first Linear
  split over ``[x || agg]`` (no concat).
* Distribution: each edge set lives with the rank that aggregates it (see
  :mod:`dgraph_amd.data.graphcast_graph`), so the only communication is one halo exchange
  of the non-aggregating endpoint's features per edge block, through the set's
  :class:`CommunicationPattern` (RCCL all-to-all-v on GPUs).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.act import linear_act
from ..ops.aggregate import scatter_sum
from ..ops.dense import linear
from ..ops.norm import layer_norm
from ..ops.csr import IndexMap
from ..ops.edge_mlp import edge_pre_activation
from ..utils.timing import region


@dataclass
class TrainingConfig:
    """graphcast_config.py:17-30."""

    lr: float = 1e-3
    lr_step3: float = 3e-7
    num_iters_step1: int = 1000
    num_iters_step2: int = 299000
    num_iters_step3: int = 11000
    step_change_freq: int = 1000
    save_freq: int = 1
    grad_clip_norm: float = 32.0
    val_freq: int = 5


@dataclass
class DataConfig:
    latlon_res: Tuple[int, int] = (721, 1440)
    num_samples_per_year_train: int = 4
    num_channels_climate: int = 73
    num_channels_static: int = 5
    num_history: int = 0
    use_cos_zenith: bool = True
    dt: float = 6.0
    start_year: int = 1980
    use_time_of_year_index: bool = True
    stride: int = 1


@dataclass
class ModelConfig:
    processor_layers: int = 4
    hidden_dim: int = 128
    mesh_level: int = 6
    multimesh: bool = True
    input_grid_dim: int = 73
    input_mesh_dim: int = 3
    input_edge_dim: int = 4
    output_grid_dim: int = 73


@dataclass
class Config:
    training: TrainingConfig = field(default_factory=TrainingConfig)
    data: DataConfig = field(default_factory=DataConfig)
    model: ModelConfig = field(default_factory=ModelConfig)


def _act_name(act: nn.Module) -> str:
    if isinstance(act, nn.SiLU):
        return "silu"
    if isinstance(act, nn.ReLU):
        return "relu"
    raise NotImplementedError(f"fused layers support SiLU/ReLU, got {act}")


class MeshGraphMLP(nn.Module):
    def __init__(self, input_dim: int, output_dim: int, hidden_dim: int = 512,
                 hidden_layers: int = 1, activation_fn: Optional[nn.Module] = None,
                 norm_type: Optional[str] = "LayerNorm"):
        super().__init__()
        self.input_dim, self.output_dim = input_dim, output_dim
        act = activation_fn if activation_fn is not None else nn.SiLU()
        layers = [nn.Linear(input_dim, hidden_dim), act]
        for _ in range(hidden_layers - 1):
            layers += [nn.Linear(hidden_dim, hidden_dim), act]
        layers.append(nn.Linear(hidden_dim, output_dim))
        if norm_type is not None:
            layers.append(getattr(nn, norm_type)(output_dim))
        self._model = nn.Sequential(*layers)

    def _run(self, h: torch.Tensor, start: int, residual=None) -> torch.Tensor:
        mods = list(self._model)[start:]
        skip = False
        for i, m in enumerate(mods):
            if skip:  # the activation already applied by linear_act
                skip = False
                continue
            if isinstance(m, nn.Linear) and i + 1 < len(mods) and \
                    isinstance(mods[i + 1], (nn.SiLU, nn.ReLU)):
                # Linear + bias + activation: one product and one fused pass each way
                h = linear_act([(h, m.weight)], m.bias, _act_name(mods[i + 1]))
                skip = True
            elif isinstance(m, nn.Linear):
                h = linear(h, m.weight, m.bias)
            elif isinstance(m, nn.LayerNorm) and i == len(mods) - 1:
                h = layer_norm(h, m.weight, m.bias, m.eps, residual)  # residual fused
                residual = None
            else:
                h = m(h)
        return h if residual is None else h + residual

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self._run(x, 0, residual)

    def tail(self, h: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Everything after the first Linear + activation (``+ residual``)."""
        return self._run(h, 2, residual)

    def first_act_name(self) -> str:
        return _act_name(self._model[1])


class MeshEdgeBlock(nn.Module):
    def __init__(self, input_src_node_dim: int, input_dst_node_dim: int, input_edge_dim: int,
                 output_edge_dim: int, comm=None, hidden_dim: int = 512,
                 num_hidden_layers: int = 1, aggregation_type: str = "sum"):
        super().__init__()
        assert aggregation_type == "sum", "Only sum aggregation is supported."
        self.comm = comm
        self.dims = (input_src_node_dim, input_dst_node_dim, input_edge_dim)
        self.mesh_mlp = MeshGraphMLP(input_src_node_dim + input_dst_node_dim + input_edge_dim,
                                     output_edge_dim, hidden_dim, num_hidden_layers)
        self._maps: dict = {}

    def _split_first(self):
        lin = self.mesh_mlp._model[0]
        a, b, _ = self.dims
        W = lin.weight
        return W[:, :a], W[:, a:a + b], W[:, a + b:], lin.bias

    def fused(self, src_feats: torch.Tensor, dst_feats: torch.Tensor, edge_feats: torch.Tensor,
              src_map: IndexMap, dst_map: IndexMap, pre=None) -> torch.Tensor:
        """Edge update with index maps over the rows of ``src_feats`` / ``dst_feats``.
        ``pre``: ``(Y, Q)`` from :meth:`pre_dst`, computed earlier (e.g. on a branch)."""
        Ws, Wd, We, b = self._split_first()
        P = linear(src_feats, Ws)
        Y, Q = pre if pre is not None else self.pre_dst(edge_feats, dst_feats)
        h = edge_pre_activation(Y, P, Q, src_map, dst_map, self.mesh_mlp.first_act_name())
        return self.mesh_mlp.tail(h, residual=edge_feats)

    def pre_dst(self, edge_feats: torch.Tensor, dst_feats: torch.Tensor):
        """The first Linear's edge term (with the bias) and destination-side projection:
        ``(edge W_e^T + b, dst W_d^T)``, which need neither the sources nor their halo."""
        _, Wd, We, b = self._split_first()
        return linear(edge_feats, We, b), linear(dst_feats, Wd)

    def fused_halo(self, src_local: torch.Tensor, dst_local: torch.Tensor,
                   edge_feats: torch.Tensor, src_map: IndexMap, dst_map: IndexMap,
                   halo, side: str, pre=None) -> torch.Tensor:
        """:meth:`fused` with one endpoint's rows ``[local | halo]`` where the halo rows are
        still on the links (``halo``: an :class:`~dgraph_amd.parallel.halo.AsyncHalo`, or
        None when the edge set has no remote endpoint): the edge GEMM, the other endpoint's
        projection and the local rows' projection run first, the exchange is waited for
        only before its rows are projected (``side`` = "src" or "dst": the halo side). The
        index maps address the projected rows ``[local | halo]`` as before."""
        if halo is None:
            return self.fused(src_local, dst_local, edge_feats, src_map, dst_map, pre)
        Ws, Wd, We, b = self._split_first()
        if side == "src":
            Y, Q = pre if pre is not None else self.pre_dst(edge_feats, dst_local)
            P_loc = linear(src_local, Ws)
            with region("exchange-wait"):  # exposed exchange time (device)
                hw = halo.wait()
            P = torch.cat([P_loc, linear(hw, Ws)], dim=0)
        else:
            assert pre is None, "pre_dst applies to a source-side halo"
            Y = linear(edge_feats, We, b)
            P = linear(src_local, Ws)
            Q_loc = linear(dst_local, Wd)
            with region("exchange-wait"):
                hw = halo.wait()
            Q = torch.cat([Q_loc, linear(hw, Wd)], dim=0)
        h = edge_pre_activation(Y, P, Q, src_map, dst_map, self.mesh_mlp.first_act_name())
        return self.mesh_mlp.tail(h, residual=edge_feats)

    def forward(self, src_node_features, dst_node_features, edge_features, src_indices,
                dst_indices, src_rank_mapping=None, dst_rank_mapping=None):
        """Reference signature (single process, global indices)."""
        key = (src_indices.data_ptr(), dst_indices.data_ptr(), src_indices.numel(),
               src_node_features.shape[0], dst_node_features.shape[0])
        maps = self._maps.get(key)
        if maps is None:
            maps = (IndexMap(src_indices.reshape(-1).long(), src_node_features.shape[0]),
                    IndexMap(dst_indices.reshape(-1).long(), dst_node_features.shape[0]))
            self._maps = {key: maps}
        return self.fused(src_node_features, dst_node_features, edge_features, *maps)


class MeshNodeBlock(nn.Module):
    def __init__(self, input_node_dim: int, input_edge_dim: int, output_node_dim: int,
                 comm=None, hidden_dim: int = 512, num_hidden_layers: int = 1,
                 aggregation_type: str = "sum"):
        super().__init__()
        assert aggregation_type == "sum", "Only sum aggregation is supported."
        self.comm = comm
        self.node_dim = input_node_dim
        self.mesh_mlp = MeshGraphMLP(input_node_dim + input_edge_dim, output_node_dim,
                                     hidden_dim, num_hidden_layers)
        self._maps: dict = {}

    def fused(self, node_features: torch.Tensor, edge_features: torch.Tensor,
              agg_map: IndexMap) -> torch.Tensor:
        agg = scatter_sum(edge_features, agg_map)
        lin = self.mesh_mlp._model[0]
        n = self.node_dim
        # the first Linear over [x || agg] as two terms of one product, bias and activation
        # fused (no concatenation, no separate add / activation passes)
        h = linear_act([(node_features, lin.weight[:, :n]),
                        (agg.to(node_features.dtype), lin.weight[:, n:])], lin.bias,
                       self.mesh_mlp.first_act_name())
        return self.mesh_mlp.tail(h, residual=node_features)

    def forward(self, node_features, edge_features, src_indices, rank_mapping=None):
        """Reference signature: edges are summed into ``node_features`` rows
        ``src_indices[e]``."""
        key = (src_indices.data_ptr(), src_indices.numel(), node_features.shape[0])
        m = self._maps.get(key)
        if m is None:
            m = IndexMap(src_indices.reshape(-1).long(), node_features.shape[0])
            self._maps = {key: m}
        return self.fused(node_features, edge_features, m)


# ----------------------------------------------------------------------------- model
class _Halo:
    """Halo exchange of an edge set's non-aggregating endpoint. ``start(x, es)``: the
    exchange issued asynchronously (:class:`~dgraph_amd.parallel.halo.AsyncHalo`; None when
    the set has no remote endpoint), consumed by :meth:`MeshEdgeBlock.fused_halo` after
    the work that does not need it. ``__call__``: the synchronous ``[local | halo]`` rows
    (the reference's form, haloExchange.py:137 + DGraphMessagePassing's concatenation)."""

    def __init__(self, comm):
        self.comm = comm
        self._ex = None

    def start(self, x: torch.Tensor, es):
        if es.pattern is None:
            return None
        from ..parallel.halo import AsyncHalo

        with region("exchange-issue"):
            return AsyncHalo.start(self.comm, x, es.pattern)

    def __call__(self, x: torch.Tensor, es) -> torch.Tensor:
        if es.pattern is None:
            return x
        if self._ex is None:
            from ..parallel.halo import HaloExchange

            self._ex = HaloExchange(self.comm)
        return torch.cat([x, self._ex(x, es.pattern)], dim=0)


class GraphCastEmbedder(nn.Module):
    def __init__(self, cfg, *args, **kwargs):
        super().__init__()
        m = cfg.model
        H = m.hidden_dim
        self.grid_input_dim, self.mesh_input_dim, self.hidden_dim = (m.input_grid_dim,
                                                                     m.input_mesh_dim, H)
        self.grid_feature_embedder = MeshGraphMLP(m.input_grid_dim, H, H, 1)
        self.mesh_feature_embedder = MeshGraphMLP(m.input_mesh_dim, H, H, 1)
        self.grid2mesh_edge_embedder = MeshGraphMLP(m.input_edge_dim, H, H, 1)
        self.mesh2grid_edge_embedder = MeshGraphMLP(m.input_edge_dim, H, H, 1)
        self.mesh2mesh_edge_embedder = MeshGraphMLP(m.input_edge_dim, H, H, 1)

    def forward(self, grid_features, mesh_features, mesh2mesh_edge_features,
                grid2mesh_edge_features, mesh2grid_edge_features):
        return (self.grid_feature_embedder(grid_features),
                self.mesh_feature_embedder(mesh_features),
                self.mesh2mesh_edge_embedder(mesh2mesh_edge_features),
                self.grid2mesh_edge_embedder(grid2mesh_edge_features),
                self.mesh2grid_edge_embedder(mesh2grid_edge_features))


class _Branch:
    """A second stream for independent parts of the step (forked from and joined into the
    current stream; autograd runs each op's backward on its forward's stream, so the
    backwards overlap too, and a HIP-graph capture records the fork and join)."""

    def __init__(self, device: torch.device):
        self.stream = torch.cuda.Stream(device)


class _on_branch:
    """``with _on_branch(branch, x) as br: y = f(x)`` runs ``f`` on the branch stream (after
    everything already issued on the current one); ``br.join(y)`` makes the current stream
    wait for that block only (an event recorded at its end: later blocks on the branch keep
    running) and returns ``y``. Without a branch both are no-ops."""

    def __init__(self, branch: Optional[_Branch], ref: torch.Tensor, reads=()):
        self.branch = branch if branch is not None and ref.is_cuda else None
        self.reads = reads
        self._ctx = None

    def __enter__(self):
        if self.branch is not None:
            self.cur = torch.cuda.current_stream()
            self.branch.stream.wait_stream(self.cur)
            for t in self.reads:  # current-stream tensors the branch reads
                t.record_stream(self.branch.stream)
            self._ctx = torch.cuda.stream(self.branch.stream)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self._ctx is not None:
            self.done = torch.cuda.Event()
            self.done.record(self.branch.stream)
            self._ctx.__exit__(*exc)
        return False

    def join(self, *ts):
        if self.branch is not None:
            self.cur.wait_event(self.done)
            for t in ts:
                t.record_stream(self.cur)  # allocated on the branch, used on the current
        return ts[0] if len(ts) == 1 else ts


class GraphCastEncoder(nn.Module):
    def __init__(self, cfg, comm=None, *args, **kwargs):
        super().__init__()
        H = cfg.model.hidden_dim
        self.edge_mlp = MeshEdgeBlock(H, H, H, H, comm, H)
        self.mesh_node_mlp = MeshNodeBlock(H, H, H, comm, H)
        self.grid_node_mlp = MeshGraphMLP(H, H)
        self.halo = _Halo(comm)

    def forward(self, grid_node_features, mesh_node_features, g2m_edge_features, g2m,
                branch: Optional["_Branch"] = None) -> Tuple:
        grid_h = self.halo.start(grid_node_features, g2m)   # senders: grid (local|halo)
        # the grid node update does not depend on the grid2mesh edges: on the branch stream
        # it runs next to the edge block and the mesh node update (and so do their backwards)
        with _on_branch(branch, grid_node_features, reads=(grid_node_features,)) as br:
            grid_out = self.grid_node_mlp(grid_node_features, residual=grid_node_features)
        e = self.edge_mlp.fused_halo(grid_node_features, mesh_node_features, g2m_edge_features,
                                     g2m.other_map(), g2m.agg_map(), grid_h, "src")
        n = self.mesh_node_mlp.fused(mesh_node_features, e, g2m.agg_map())
        mesh_node_features = mesh_node_features + n
        return br.join(grid_out), mesh_node_features


class GraphCastProcessor(nn.Module):
    def __init__(self, cfg, comm=None, *args, **kwargs):
        super().__init__()
        H = cfg.model.hidden_dim
        L = cfg.model.processor_layers
        self.edge_processors = nn.ModuleList([MeshEdgeBlock(H, H, H, H, comm, H)
                                              for _ in range(L)])
        self.node_processors = nn.ModuleList([MeshNodeBlock(H, H, H, comm, H)
                                              for _ in range(L)])
        self.halo = _Halo(comm)

    def forward(self, mesh_features, m2m_edge_features, m2m) -> Tuple:
        e, n = m2m_edge_features, mesh_features
        for i, (el, nl) in enumerate(zip(self.edge_processors, self.node_processors)):
            with region(f"processor-{i}"):
                n_h = self.halo.start(n, m2m)        # receivers (dst) may be remote
                e = el.fused_halo(n, n, e, m2m.agg_map(), m2m.other_map(), n_h, "dst")
                n = nl.fused(n, e, m2m.agg_map())    # aggregate at the source
        return n, e


class GraphCastDecoder(nn.Module):
    def __init__(self, cfg, comm=None, *args, **kwargs):
        super().__init__()
        H = cfg.model.hidden_dim
        self.comm = comm
        self.edge_mlp = MeshEdgeBlock(H, H, H, H, comm, H)
        self.node_mlp = MeshNodeBlock(H, H, H, comm, H, 1)
        self.halo = _Halo(comm)

    def forward(self, m2g_edge_features, grid_node_features, mesh_node_features, m2g):
        mesh_h = self.halo.start(mesh_node_features, m2g)  # senders: mesh (local|halo)
        e = self.edge_mlp.fused_halo(mesh_node_features, grid_node_features,
                                     m2g_edge_features, m2g.other_map(), m2g.agg_map(),
                                     mesh_h, "src")
        n = self.node_mlp.fused(grid_node_features, e, m2g.agg_map())
        return grid_node_features + n


class DGraphCast(nn.Module):
    def __init__(self, cfg, comm=None, *args, **kwargs):
        super().__init__()
        self.hidden_dim = cfg.model.hidden_dim
        self.output_grid_dim = cfg.model.output_grid_dim
        self.comm = comm
        self.embedder = GraphCastEmbedder(cfg)
        self.encoder = GraphCastEncoder(cfg, comm)
        self.processor = GraphCastProcessor(cfg, comm)
        self.decoder = GraphCastDecoder(cfg, comm)
        self.final_prediction = MeshGraphMLP(self.hidden_dim, self.output_grid_dim)
        # independent parts on a second stream (GPU): the mesh2grid edge embedding next to
        # the encoder and the processor (whose mesh-sized kernels fill a fraction of the
        # CUs), the encoder's grid node update next to its edge block
        self.branch_streams = True
        self._branch: Optional[_Branch] = None

    def forward(self, input_grid_features: torch.Tensor, static_graph) -> torch.Tensor:
        g = static_graph
        x = input_grid_features.reshape(-1, input_grid_features.shape[-1])
        br = None
        if self.branch_streams and x.is_cuda:
            if self._branch is None or self._branch.stream.device != x.device:
                self._branch = _Branch(x.device)
            br = self._branch
        emb = self.embedder
        with region("embedder"):
            # the mesh2grid edge embedding (first used by the decoder) on the branch; the
            # branch stays short ahead of the encoder's grid update, which joins at the
            # encoder's end (measured: also moving the mesh and multimesh embeddings there
            # delayed that join, W=8 rank 0 15.96 -> 16.86 ms)
            with _on_branch(br, x) as m2g_branch:
                e_m2g = emb.mesh2grid_edge_embedder(g.m2g.features.to(x.dtype))
            grid = emb.grid_feature_embedder(x)
            mesh = emb.mesh_feature_embedder(g.mesh_node_features.to(x.dtype))
            e_m2m = emb.mesh2mesh_edge_embedder(g.m2m.features.to(x.dtype))
            e_g2m = emb.grid2mesh_edge_embedder(g.g2m.features.to(x.dtype))
        with region("encoder"):
            grid, mesh = self.encoder(grid, mesh, e_g2m, g.g2m, branch=br)
        # (the decoder's edge / grid projections, MeshEdgeBlock.pre_dst, were also tried on
        # the branch beside the processor: slower, W=8 rank 0 15.96 -> 16.34 ms)
        with region("processor"):
            mesh, _ = self.processor(mesh, e_m2m, g.m2m)
        e_m2g = m2g_branch.join(e_m2g)
        with region("decoder"):
            grid = self.decoder(e_m2g, grid, mesh, g.m2g)
        with region("final"):
            return self.final_prediction(grid)
