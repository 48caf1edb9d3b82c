"""Environment check, plan statistics / validation and comm fault injection (CPU)."""
import pytest
import torch

from dgraph_amd.comm.alltoallv import AllToAllV
from dgraph_amd.comm.faults import FaultInjector, InjectedFault, parse, set_fault
from dgraph_amd.ops.csr import CSR
from dgraph_amd.parallel.dist_graph import DistGraph
from dgraph_amd.utils import diagnostics as D


def _ring_graph(L=10, halo=0):
    rows = torch.arange(L).repeat_interleave(2)
    cols = torch.stack([(torch.arange(L) + 1) % L, (torch.arange(L) - 1) % L], 1).reshape(-1)
    return CSR.from_coo(rows, cols, L, L + halo)


def test_env_check_reports_fields():
    rep = D.env_check(verbose=False)
    for k in ("rocm_path", "torch", "gpu_count", "native_lib", "problems"):
        assert k in rep
    assert isinstance(rep["problems"], list)


def test_validate_graph_accepts_and_rejects():
    g = DistGraph(_ring_graph(), 10, 0)
    D.validate_graph(g)
    bad = _ring_graph()
    bad.col[3] = 57  # out of range
    with pytest.raises(D.PlanError):
        D.validate_graph(DistGraph(bad, 10, 0))


def test_check_plans_env_validates_at_construction(monkeypatch):
    monkeypatch.setenv("DGRAPH_CHECK_PLANS", "1")
    bad = _ring_graph()
    bad.rowptr[4] = bad.rowptr[6] + 1  # non-monotone
    with pytest.raises(D.PlanError):
        DistGraph(bad, 10, 0)


def test_fault_rules_parse_and_apply():
    rules = parse("delay:ms=1:rank=0;corrupt:call=2;fail:rank=3")
    assert [r.kind for r in rules] == ["delay", "corrupt", "fail"]
    with pytest.raises(ValueError):
        parse("explode")
    a2a = AllToAllV([4], [4])
    x = torch.ones(4, 3)
    try:
        set_fault("corrupt:call=2")
        assert torch.equal(a2a(x), x)            # call 1: untouched
        assert torch.count_nonzero(a2a(x)) == 0  # call 2: zeroed payload
        set_fault("fail:call=1")
        with pytest.raises(InjectedFault):
            a2a(x)
        assert FaultInjector.log == ["fail@rank0/call1"]
    finally:
        set_fault(None)
    assert not FaultInjector.active()


def _straggler_and_stats(rank, world):
    import torch.distributed as dist

    from dgraph_amd.comm.faults import set_fault

    # each rank sends its rank id to every peer; rank 1 is delayed but results hold
    set_fault("delay:ms=50:rank=1")
    a2a = AllToAllV([1] * world, [1] * world)
    out = a2a(torch.full((world, 2), float(rank)))
    assert out[:, 0].tolist() == [float(r) for r in range(world)]
    set_fault(None)

    class _G:  # minimal graph view for halo_stats
        L, H = 5, world - 1
        device = torch.device("cpu")

    _G.a2a = AllToAllV([0 if p == rank else rank + 1 for p in range(world)],
                       [0 if p == rank else p + 1 for p in range(world)])
    st = D.halo_stats(_G, feature_bytes=512)
    assert st["max_peer_bytes_local"] == (rank + 1) * 512
    assert st["max_pairwise_bytes"] == world * 512
    assert st["xgmi_bound_ms"] > 0
    dist.barrier()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_straggler_exchange_and_halo_stats(ranks, world):
    ranks(_straggler_and_stats, world)


def test_plot_timing_reports(tmp_path):
    import json
    import subprocess
    import sys

    for w in (1, 2):
        with open(tmp_path / f"arxiv_timing_report_world{w}.json", "w") as f:
            json.dump({"halo": [9.0, 1.0 * w, 1.0 * w], "compute": [9.0, 3.0, 3.0]}, f)
    out = tmp_path / "t.png"
    r = subprocess.run([sys.executable, "scripts/plot_timing_reports.py", "--log-dir",
                        str(tmp_path), "--dataset", "arxiv", "--out", str(out)],
                       capture_output=True, text=True, cwd=D.__file__.rsplit("/dgraph_amd/", 1)[0])
    assert r.returncode == 0, r.stderr
    assert out.exists() and "compute" in r.stdout
