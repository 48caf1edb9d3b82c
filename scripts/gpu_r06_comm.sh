#!/bin/bash
# Round 6, first GPU call: the comm-path GPU tests (multi-device ones skip on one GPU) and
# bench.py at W=2 / W=8 with every rank on the one GPU (RCCL socket transport), whose JSON
# line now carries the one-sided probe child job's record (mode: host on a shared GPU).
set -o pipefail
mkdir -p gpurun_out/r06
cd /root/repo
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_multidevice_gpu.py tests/test_comm_native_gpu.py tests/test_rccl_gpu.py \
  tests/test_multiproc_gpu.py > gpurun_out/r06/gpu_comm_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06/gpu_comm_tests.log; exit 1; }
tail -3 gpurun_out/r06/gpu_comm_tests.log
DGRAPH_RCCL_SHARED_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --scale 0.02 --steps 2 \
  --warmup 1 --no-extra > gpurun_out/r06/bench_w2_shared.json 2> gpurun_out/r06/bench_w2_shared.err \
  || { echo "w2 bench failed"; tail -30 gpurun_out/r06/bench_w2_shared.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06/bench_w2_shared.json').read().splitlines()[-1]);print(json.dumps(d['shmem_probe']))"
DGRAPH_RCCL_SHARED_GPU=1 timeout -k 10 500 python -u bench.py --gpus 8 --scale 0.02 --steps 2 \
  --warmup 1 --no-extra > gpurun_out/r06/bench_w8_shared.json 2> gpurun_out/r06/bench_w8_shared.err \
  || { echo "w8 bench failed"; tail -30 gpurun_out/r06/bench_w8_shared.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06/bench_w8_shared.json').read().splitlines()[-1]);print(json.dumps(d['shmem_probe']))"
