set -o pipefail
mkdir -p gpurun_out/colsum
timeout -k 10 500 python -u -m pytest tests/test_row_scale_colsum_gpu.py tests/test_kernels_gpu.py tests/test_precision_gpu.py tests/test_determinism.py tests/test_halo_recompute_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/colsum/pytest.log 2>&1 || { tail -30 gpurun_out/colsum/pytest.log; exit 1; }
tail -1 gpurun_out/colsum/pytest.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-extra > gpurun_out/colsum/bench.log 2>&1 || { tail -20 gpurun_out/colsum/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/colsum/bench.log | head -1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --rehearse-world 2 --rehearse-rank 1 > gpurun_out/colsum/reh2.log 2>&1 || { tail -20 gpurun_out/colsum/reh2.log; exit 1; }
grep '^{' gpurun_out/colsum/reh2.log
