# round 6: the at-size tests (config 4's rank shape with and without the
# exchange, the G = 8 multi-GB simulated ranks, config 5 at 3.1 Gbp)
set -e
TAG=${1:-r06a}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu -x \
  tests/test_gpu_atsize.py tests/test_gpu_config4.py --durations=0 > gpurun_out/atsize_$TAG.log 2>&1 \
  || { tail -60 gpurun_out/atsize_$TAG.log; exit 1; }
tail -30 gpurun_out/atsize_$TAG.log
