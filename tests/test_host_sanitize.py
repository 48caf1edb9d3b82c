"""Native host code under CPU sanitizers (GPU ASan is not available on the
target pool, so the host-side plan checks are built and run under ASan+UBSan and TSan) and
the same checks reached through the library (DGRAPH_CHECK_PLANS=1 path)."""
import os
import shutil
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None,
                    reason="needs g++ and make")
def test_plan_checks_under_asan_ubsan_and_tsan(tmp_path):
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "csrc", "host"), f"OUT={tmp_path}",
                        "test", "sanitize"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("plan_check host tests passed") == 3


def _ops():
    from dgraph_amd import _native

    if not _native.load():
        pytest.skip("native library not built")
    return _native.ops()


def test_native_validators_through_bindings():
    ops = _ops()
    rp = torch.tensor([0, 2, 3, 5])
    col = torch.tensor([0, 4, 1, 2, 3], dtype=torch.int32)
    ops.validate_csr(rp, col, 5)
    with pytest.raises(RuntimeError, match="column id out of range"):
        ops.validate_csr(rp, col, 4)
    ops.validate_row_map(torch.tensor([3, 0, 2]), 4)
    with pytest.raises(RuntimeError, match="write race"):
        ops.validate_row_map(torch.tensor([3, 0, 3]), 4)
    ops.validate_splits(torch.tensor([1, 2]), torch.tensor([0, 4]), 3, 4)
    with pytest.raises(RuntimeError, match="recv splits"):
        ops.validate_splits(torch.tensor([1, 2]), torch.tensor([0, 4]), 3, 5)


def test_validate_graph_checks_compact_and_hub_caches():
    from dgraph_amd.ops.csr import CSR
    from dgraph_amd.utils.diagnostics import PlanError, _check_csr

    _ops()
    g = torch.Generator().manual_seed(0)
    rows = torch.cat([torch.zeros(300, dtype=torch.long), torch.randint(1, 50, (200,), generator=g)])
    cols = torch.randint(0, 60, (500,), generator=g)
    csr = CSR.from_coo(rows, cols, 50, 60)
    csr.hub_split(64)
    csr.compact_rows()
    _check_csr(csr, "t", 50, 60)  # valid
    csr._compact.row_map[1] = csr._compact.row_map[0]
    with pytest.raises(PlanError, match="write race"):
        _check_csr(csr, "t", 50, 60)
