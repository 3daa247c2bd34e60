# A/B of the digit pass: HEAD build (kman_amd/lib_abl_head) vs the working tree, shapes given
set -e
mkdir -p gpurun_out
KMAN_RG_PASS=${TEST_SHAPE:-7} timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for i in 1 2; do
KMAN_LIB=kman_amd/lib_abl_head/libkman.so timeout -k 10 200 python -u tools/regionbench.py uniq ${HEAD_CFG:-KMAN_RG_PASS=7:0} 2>&1 | sed 's/^/head /'
timeout -k 10 200 python -u tools/regionbench.py uniq ${NEW_CFG:-KMAN_RG_PASS=5:0,KMAN_RG_PASS=7:0} 2>&1 | sed 's/^/new  /'
done | tee gpurun_out/ab.log
