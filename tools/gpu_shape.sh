# digit-pass block shapes (KMAN_RG_PASS = 0, 1, 2): parity, then stage times
set -e
mkdir -p gpurun_out
KMAN_RG_PASS=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py -x -q --timeout 300 --timeout-method thread > gpurun_out/shape_tests.log 2>&1 || { tail -40 gpurun_out/shape_tests.log; exit 1; }
tail -2 gpurun_out/shape_tests.log
timeout -k 10 300 python -u tools/regionbench.py uniq KMAN_RG_PASS=0:0,KMAN_RG_PASS=1:0,KMAN_RG_PASS=2:0,KMAN_RG_PASS=0:0,KMAN_RG_PASS=2:0 2>&1 | tee gpurun_out/shape.log
KMAN_LIB=kman_amd/lib_abl_pabl/libkman.so timeout -k 10 300 python -u tools/regionbench.py uniq KMAN_RG_PASS=2:0,KMAN_RG_PASS=2:64,KMAN_RG_PASS=2:128,KMAN_RG_PASS=0:0,KMAN_RG_PASS=0:64,KMAN_RG_PASS=0:128 2>&1 | tee -a gpurun_out/shape.log
