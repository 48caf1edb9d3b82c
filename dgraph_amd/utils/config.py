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
    dtype: str = "bf16"


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
class RunConfig:
    comm: CommConfig = field(default_factory=CommConfig)
    kernels: KernelConfig = field(default_factory=KernelConfig)
    model: ModelConfig = field(default_factory=ModelConfig)
    train: TrainConfig = field(default_factory=TrainConfig)
    data: DataConfig = field(default_factory=DataConfig)

    @staticmethod
    def from_env(environ=None) -> "RunConfig":
        cfg = RunConfig()
        env = os.environ if environ is None else environ
        for sec in dataclasses.fields(cfg):
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
        return v.strip().lower() in ("1", "true", "yes", "on")
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
    return cfg


def clear_buffer_cache_enabled() -> bool:
    return os.environ.get("DGRAPH_CLEAR_BUFFER_CACHE", "0") == "1"
