# GPU call: the multi-GPU path tests (SimGroup + RCCL world 1), then the full suite
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1 || { tail -60 gpurun_out/pytest_dist.log; exit 1; }
tail -3 gpurun_out/pytest_dist.log
