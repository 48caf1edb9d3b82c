"""Environment checks, plan statistics and plan validation.

* :func:`env_check` — the MI355X counterpart of the reference's NVSHMEM pre-install check
  (experiments/NVSHMEM-Enabled-DGRAPH/PreInstallCheck.py:19-134): ROCm toolchain, device
  architecture, RCCL, the IPC mode the symmetric heap needs, the native op library.
* :func:`halo_stats` — per-peer halo volume of a :class:`DistGraph` and the xGMI time it
  implies (the max pairwise volume bounds an all-to-all-v on a point-to-point mesh, not
  the total; §5.8), the ``dump_plan_stats`` of §5.1 (printed by setup_dataset_comms.py in
  the reference).
* :func:`validate_graph` — index-bounds / ordering / split-consistency checks run ONCE per
  plan when ``DGRAPH_CHECK_PLANS=1`` (replaces the per-call ``.max().item()`` asserts of
  RankLocalOps.py:183-184, which cost a device sync every call).
"""
from __future__ import annotations

import os
import shutil
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

XGMI_LINK_GBPS = 153.0  # per direction, per link (7 links per MI355X)


def env_check(verbose: bool = True) -> Dict[str, object]:
    """Collect (and optionally print) the facts a multi-GPU run depends on."""
    rep: Dict[str, object] = {}
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    rep["rocm_path"] = rocm if os.path.isdir(rocm) else None
    rep["hipcc"] = shutil.which("hipcc") or (os.path.join(rocm, "bin", "hipcc")
                                             if os.path.exists(os.path.join(rocm, "bin", "hipcc"))
                                             else None)
    rep["torch"] = torch.__version__
    rep["torch_hip"] = getattr(torch.version, "hip", None)
    try:
        rep["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
    except Exception:  # noqa: BLE001 - absent on CPU-only builds
        rep["rccl_version"] = None
    rep["ipc_mode_legacy"] = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    rep["ipc_ok_for_symheap"] = rep["ipc_mode_legacy"] == "0"
    rep["gpu_count"] = torch.cuda.device_count()
    archs: List[str] = []
    if torch.cuda.is_available():
        for i in range(torch.cuda.device_count()):
            p = torch.cuda.get_device_properties(i)
            archs.append(getattr(p, "gcnArchName", p.name))
        rep["hbm_gb"] = [round(torch.cuda.get_device_properties(i).total_memory / 2**30, 1)
                         for i in range(torch.cuda.device_count())]
    rep["archs"] = archs
    rep["gfx950"] = all(a.startswith("gfx950") for a in archs) if archs else None
    from .. import _native

    rep["native_lib"] = _native.library_path() if _native.available() else None
    rep["dist_initialized"] = dist.is_available() and dist.is_initialized()
    problems = []
    if rep["rocm_path"] is None:
        problems.append("ROCm not found (set ROCM_PATH)")
    if archs and not rep["gfx950"]:
        problems.append(f"device arch {archs} is not gfx950: the native kernels target gfx950")
    if torch.cuda.device_count() > 1 and not rep["ipc_ok_for_symheap"]:
        problems.append("HSA_ENABLE_IPC_MODE_LEGACY != 0: RCCL / symmetric-heap IPC needs dmabuf")
    if rep["native_lib"] is None:
        problems.append("native library dgraph_amd/_C.so not built (python -m dgraph_amd._build)")
    rep["problems"] = problems
    if verbose:
        for k, v in rep.items():
            print(f"{k:20s} {v}")
    return rep


def halo_stats(graph, feature_bytes: int, group=None) -> Dict[str, object]:
    """Halo volume of one exchange of ``feature_bytes`` per row through ``graph``'s plan.

    Returns per-peer send/recv rows and bytes of this rank, and (collectively, when a
    process group is up) the max pairwise volume over all ranks with the xGMI time bound
    ``max_bytes / 153 GB/s``."""
    a2a = getattr(graph, "a2a", None)
    send = list(a2a.send_splits) if a2a is not None else [0]
    recv = list(a2a.recv_splits) if a2a is not None else [0]
    out: Dict[str, object] = {
        "num_local": int(graph.L), "num_halo": int(graph.H),
        "send_rows_per_peer": send, "recv_rows_per_peer": recv,
        "send_bytes": sum(send) * feature_bytes, "recv_bytes": sum(recv) * feature_bytes,
        "max_peer_bytes_local": max(send + [0]) * feature_bytes,
    }
    if dist.is_available() and dist.is_initialized() and len(send) > 1:
        dev = graph.device if graph.device.type == "cuda" else torch.device("cpu")
        t = torch.tensor([out["max_peer_bytes_local"], out["send_bytes"]],
                         dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        out["max_pairwise_bytes"] = float(t[0])
        out["max_rank_send_bytes"] = float(t[1])
        out["xgmi_bound_ms"] = float(t[0]) / (XGMI_LINK_GBPS * 1e9) * 1e3
    return out


class PlanError(ValueError):
    pass


def _native_ops():
    """The native host checkers (csrc/host/plan_check.cpp) when the library is loaded."""
    try:
        from .. import _native

        if _native.load():
            ops = _native.ops()
            return ops if hasattr(ops, "validate_csr") else None
    except Exception:  # noqa: BLE001 - fall back to the torch checks
        pass
    return None


def _raise_native(fn, *args) -> None:
    try:
        fn(*args)
    except RuntimeError as e:
        raise PlanError(str(e).split("\n")[0]) from None


def _check_csr(csr, name: str, num_rows: int, num_cols: int) -> None:
    rp, col = csr.rowptr, csr.col
    if rp.numel() != num_rows + 1:
        raise PlanError(f"{name}: rowptr has {rp.numel()} entries, expected {num_rows + 1}")
    ops = _native_ops()
    if ops is not None:  # multi-threaded host scan (and the sanitized code path)
        _raise_native(ops.validate_csr, rp, col, int(num_cols))
    else:
        if int(rp[0]) != 0 or int(rp[-1]) != col.numel():
            raise PlanError(f"{name}: rowptr must start at 0 and end at nnz={col.numel()}")
        if rp.numel() > 1 and bool((rp[1:] < rp[:-1]).any()):
            raise PlanError(f"{name}: rowptr is not monotone")
        if col.numel():
            lo, hi = int(col.min()), int(col.max())
            if lo < 0 or hi >= num_cols:
                raise PlanError(f"{name}: column ids span [{lo}, {hi}], outside [0, {num_cols})")
    _check_derived(csr, name, num_rows, ops)


def _check_derived(csr, name: str, num_rows: int, ops) -> None:
    """Row-compacted copies (row_map: a duplicated output row would be a write race) and
    hub splits (segments must tile each hub row exactly) cached on ``csr``."""
    comp = getattr(csr, "_compact", None)
    if comp is not None and comp.row_map is not None:
        rm = comp.row_map
        if ops is not None:
            _raise_native(ops.validate_row_map, rm, int(num_rows))
        elif rm.numel():
            if int(rm.min()) < 0 or int(rm.max()) >= num_rows:
                raise PlanError(f"{name}: row_map outside [0, {num_rows})")
            if torch.unique(rm).numel() != rm.numel():
                raise PlanError(f"{name}: row_map repeats an output row (write race)")
    hub = getattr(csr, "_hub", None)
    hub = hub[1] if hub else None  # cached as (cap, HubSplit or None)
    if hub is not None and ops is not None and hub.num_segments:
        # hub_rows are OUTPUT rows; the segments index this CSR's rows
        rows = torch.nonzero(csr.degree() > hub.cap).reshape(-1)
        out = rows if csr.row_map is None else csr.row_map[rows]
        if not torch.equal(out.cpu().long(), hub.hub_rows.cpu().long()):
            raise PlanError(f"{name}: hub rows do not match the rows longer than {hub.cap}")
        seg_row = torch.repeat_interleave(rows.long(),
                                          (hub.hub_seg_ptr[1:] - hub.hub_seg_ptr[:-1]).long())
        _raise_native(ops.validate_hub_split, csr.rowptr, seg_row, hub.seg_beg, hub.seg_end,
                      int(hub.cap))


def validate_graph(graph) -> None:
    """Check a :class:`~dgraph_amd.parallel.dist_graph.DistGraph`'s CSR blocks and halo
    plan (index bounds, ordering, split sums). Raises :class:`PlanError`."""
    L, H = int(graph.L), int(graph.H)
    _check_csr(graph.interior, "interior", L, L if graph.halo is not None else
               graph.interior.num_cols)
    if graph.halo is not None:
        _check_csr(graph.halo, "halo", L, H)
        idx = graph.send_map.idx
        if idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= L):
            raise PlanError("send_local_idx points outside the local vertices")
        if graph.a2a.total_recv != H:
            raise PlanError(f"recv splits sum {graph.a2a.total_recv} != halo rows {H}")
        if graph.a2a.total_send != idx.numel():
            raise PlanError(f"send splits sum {graph.a2a.total_send} != {idx.numel()} rows")
        ops = _native_ops()
        if ops is not None:
            _raise_native(ops.validate_splits, torch.tensor(list(graph.a2a.send_splits)),
                          torch.tensor(list(graph.a2a.recv_splits)), idx.numel(), H)
        if dist.is_available() and dist.is_initialized():
            # every peer's send count to me equals my recv count from it
            dev = idx.device if idx.is_cuda else torch.device("cpu")
            mine = torch.tensor(graph.a2a.send_splits, dtype=torch.long, device=dev)
            got = torch.empty_like(mine)
            dist.all_to_all_single(got, mine, group=graph.a2a.group)
            if got.tolist() != list(graph.a2a.recv_splits):
                raise PlanError(f"peers send {got.tolist()} rows, plan expects "
                                f"{list(graph.a2a.recv_splits)}")


def checks_enabled() -> bool:
    return os.environ.get("DGRAPH_CHECK_PLANS", "0") not in ("", "0", "false", "False")


def maybe_validate(graph) -> None:
    if checks_enabled():
        validate_graph(graph)


def main(argv: Optional[List[str]] = None) -> int:
    rep = env_check(verbose=True)
    if rep["problems"]:
        print("PROBLEMS:")
        for p in rep["problems"]:
            print("  -", p)
        return 1
    print("environment OK")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
