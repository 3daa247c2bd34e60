# round 6: every multi-GPU-path GPU test (dist, dist_region, atsize, config4)
set -e
TAG=${1:-r06y}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu -x \
  tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_atsize.py tests/test_gpu_config4.py \
  > gpurun_out/dist_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/dist_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/dist_tests_$TAG.log
