set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/region_tests.log 2>&1 || { tail -60 gpurun_out/region_tests.log; exit 1; }
tail -3 gpurun_out/region_tests.log
timeout -k 10 300 python tools/regionbench.py uniq 0,1,2,0
