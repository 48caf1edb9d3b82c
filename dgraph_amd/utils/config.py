"""One dataclass config tree with CLI and ``DGRAPH_*`` environment overrides (§5.6).

The reference spread configuration over python-fire signatures, ad-hoc dataclasses and
undocumented environment variables. Here :class:`RunConfig` gathers the knobs the library
reads; ``RunConfig.from_env()`` applies ``DGRAPH_<SECTION>_<FIELD>`` overrides and
``apply_overrides(cfg, ["comm.overlap=false", ...])`` applies ``key=value`` strings.
Recognised legacy variables: ``DGRAPH_CLEAR_BUFFER_CACHE`` (empty the caching allocator
after each comm op, _torch_func_impl.py:22).
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Any, List


@dataclass
class CommConfig:
    backend: str = "nccl"
    overlap: bool = True            # interior SpMM || halo all-to-all-v
    ranks_per_graph: int = -1       # hybrid graph-group x data-parallel
    timeout_s: int = 1800
    shmem_transport: str = "auto"   # auto | ipc | two_sided


@dataclass
class KernelConfig:
    spmm_variant: int = 4
    spmm_row_map: int = 0  # 0 grid-stride / in-order, 1-2 XCD-chunked, 3 in-order (v2)
    spmm_pass_cols: int = 128
    spmm_hub_cap: int = 2048        # hub-row split degree (0: off)
    dual_gemm_variant: int = 2      # 1 column-half (B^T in LDS), 2 B-stationary
    halo_chunk_bytes: int = 32 << 20  # per-peer message size that triggers chunking
    deterministic: bool = True      # segment sums only, no float atomics


@dataclass
class ModelConfig:
    name: str = "sage"
    hidden: int = 256
    num_layers: int = 3
    dropout: float = 0.0
    dtype: str = "fp32"  # the reference's precision (bf16 is a labelled secondary)


@dataclass
class TrainConfig:
    epochs: int = 10
    lr: float = 1e-3
    weight_decay: float = 0.0
    seed: int = 0
    log_dir: str = "logs"
    checkpoint_dir: str = ""
    checkpoint_every: int = 0


@dataclass
class DataConfig:
    dataset: str = "ogbn-arxiv"
    partition: str = "contiguous"
    scale: float = 1.0
    global_frac: float = 0.05


@dataclass
class ExecutorConfig:
    """Schedule knobs of the fp32 row-chunked executor (models/sage_fused.py FusedSAGE),
    resolved when an executor is CONSTRUCTED (not frozen at import): environment
    ``DGRAPH_FUSED_<FIELD>`` (e.g. DGRAPH_FUSED_HALO_STREAM=on), or pass an instance.
    "auto" choices are made by the executor's memory / link planner; the resolved set and
    the derived schedule are both recorded in bench.py's JSON line. Field meanings are
    documented where they are used (sage_fused.py); the reference has no executor, its
    equivalents are the experiment configs (experiments/OGB-LSC/config.py:18-45)."""
    chunk_rows: int = 0             # rows per chunk (0: from free memory)
    overlap: bool = True            # W>1: interior rows while the forward exchange flies
    keep_agg0: str = "auto"         # keep mean_N(x) for the backward: auto | on | off
    boundary_store: str = "auto"    # boundary rows' interior part pre-aggregated: auto|on|off
    keep_as: str = "auto"           # keep the S rows' last-hidden aggregate: auto|on|off
    stream_fill: bool = True        # streamed layers: self term during the first block
    stream_ramp: bool = False       # streamed halos: half-width first column block
    stream_out_fill: bool = False   # streamed output layer: self term as the pipeline fill
    halo_stream: str = "auto"       # hidden halos in column blocks: auto | on | off
    compact_t: str = "off"          # S-compacted transposed adjacency: auto | on | off
    compact_pull: str = "auto"      # pulled halo's adjacency, map applied (auto: streamed)
    pack_stream: str = "compute"    # halo pack on the compute or the comm stream
    pack_fused: bool = True         # halo pack fused into the producing GEMM's epilogue
    bwd_halo: str = "pull"          # input-layer backward halo: pull | push
    project_first: str = "auto"     # W>1 output layer projected before aggregation
    u_full_frac: float = 0.35       # full-width gradient passes while |S|/L <= this
    stream_shapes: str = "64x2,32x2,64x1,32x1"  # (column block x ring buffers), preferred first
    pass_cols: int = 0              # force the SpMM column-pass width (0: from locality)
    plan_link_gbps: float = 0.0     # planner's per-link rate (0: measured at setup)

    def __post_init__(self):
        for name, ok in (("keep_agg0", ("auto", "on", "off")),
                         ("boundary_store", ("auto", "on", "off")),
                         ("keep_as", ("auto", "on", "off")),
                         ("halo_stream", ("auto", "on", "off")),
                         ("compact_t", ("auto", "on", "off")),
                         ("compact_pull", ("auto", "on", "off")),
                         ("pack_stream", ("compute", "comm")),
                         ("bwd_halo", ("pull", "push")),
                         ("project_first", ("auto", "on", "off"))):
            if getattr(self, name) not in ok:
                raise ValueError(f"ExecutorConfig.{name}={getattr(self, name)!r}: one of {ok}")
        self.shapes()  # parse check

    def shapes(self):
        """``stream_shapes`` as ((column block, ring buffers), ...)."""
        return tuple(tuple(int(v) for v in t.split("x")) for t in self.stream_shapes.split(","))

    @staticmethod
    def from_env(environ=None) -> "ExecutorConfig":
        env = os.environ if environ is None else environ
        cfg = ExecutorConfig.__new__(ExecutorConfig)
        for f in dataclasses.fields(ExecutorConfig):
            setattr(cfg, f.name, f.default)
        for f in dataclasses.fields(cfg):
            key = f"DGRAPH_FUSED_{f.name.upper()}"
            if key in env:
                setattr(cfg, f.name, _coerce(env[key], f.type, getattr(cfg, f.name)))
        if "DGRAPH_PLAN_LINK_GBPS" in env and "DGRAPH_FUSED_PLAN_LINK_GBPS" not in env:
            cfg.plan_link_gbps = float(env["DGRAPH_PLAN_LINK_GBPS"])  # legacy name
        cfg.__post_init__()
        return cfg


@dataclass
class RunConfig:
    comm: CommConfig = field(default_factory=CommConfig)
    kernels: KernelConfig = field(default_factory=KernelConfig)
    fused: ExecutorConfig = field(default_factory=ExecutorConfig)
    model: ModelConfig = field(default_factory=ModelConfig)
    train: TrainConfig = field(default_factory=TrainConfig)
    data: DataConfig = field(default_factory=DataConfig)

    @staticmethod
    def from_env(environ=None) -> "RunConfig":
        cfg = RunConfig()
        env = os.environ if environ is None else environ
        cfg.fused = ExecutorConfig.from_env(env)
        for sec in dataclasses.fields(cfg):
            if sec.name == "fused":
                continue
            obj = getattr(cfg, sec.name)
            for f in dataclasses.fields(obj):
                key = f"DGRAPH_{sec.name.upper()}_{f.name.upper()}"
                if key in env:
                    setattr(obj, f.name, _coerce(env[key], f.type, getattr(obj, f.name)))
        return cfg

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    def apply(self) -> "RunConfig":
        """Push the kernel settings into the native library."""
        from .. import _native

        from ..parallel import dist_graph

        if _native.available():
            _native.ops().set_spmm_config(self.kernels.spmm_variant,
                                          self.kernels.spmm_row_map,
                                          self.kernels.spmm_pass_cols)
            _native.ops().set_dual_gemm_variant(self.kernels.dual_gemm_variant)
        dist_graph.SPMM_HUB_CAP = int(self.kernels.spmm_hub_cap)
        os.environ["DGRAPH_HALO_CHUNK_BYTES"] = str(int(self.kernels.halo_chunk_bytes))
        os.environ["DGRAPH_SHMEM_TRANSPORT"] = self.comm.shmem_transport
        return self


def _coerce(v: str, typ: Any, current: Any):
    if isinstance(current, bool):
        return v.strip().lower() not in ("0", "false", "no", "off", "")
    if isinstance(current, int):
        return int(v)
    if isinstance(current, float):
        return float(v)
    return v


def apply_overrides(cfg: RunConfig, overrides: List[str]) -> RunConfig:
    for item in overrides:
        key, _, val = item.partition("=")
        sec, _, name = key.partition(".")
        obj = getattr(cfg, sec)
        setattr(obj, name, _coerce(val, None, getattr(obj, name)))
    cfg.fused.__post_init__()
    return cfg


def clear_buffer_cache_enabled() -> bool:
    return os.environ.get("DGRAPH_CLEAR_BUFFER_CACHE", "0") == "1"
