"""benchmarks/bench_comm.py at W=2 (gloo, CPU): the two-sided G1 ops with and without a
cache, the halo exchange, the all-to-all-v sweep, and the one-sided backend
(``--backend rocshmem``) writing the reference's NVSHMEM_{op}_times_{rank}.npy files
(experiments/Benchmarks/TestNVSHMEM.py:160-190)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("backend,ops,files", [
    ("nccl", "gather,scatter,halo,a2a", ["NCCL_gather", "NCCL_scatter_with_cache", "NCCL_halo"]),
    ("rocshmem", "gather,scatter", ["NVSHMEM_gather", "NVSHMEM_scatter"]),
])
def test_bench_comm_two_ranks(tmp_path, backend, ops, files):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(REPO, "benchmarks", "bench_comm.py"), "--device", "cpu",
           "--iters", "4", "--warmup", "1", "--impl", "torch", "--sizes", "4096",
           "--backend", backend, "--pg-backend", "gloo", "--ops", ops,
           "--log-dir", str(tmp_path)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["world_size"] == 2 and rec["backend"] == backend
    for f in files:
        for rank in (0, 1):
            t = np.load(tmp_path / f"{f}_times_{rank}.npy")
            assert t.shape == (4,) and (t > 0).all()
