set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench1.log 2>&1 && echo BENCH_OK
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ -f gpurun_out/bench1.log ] && tail -2 gpurun_out/bench1.log
exit $rc
