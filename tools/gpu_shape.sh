# digit-pass block shapes (KMAN_RG_PASS): parity of the given shapes, then stage times
set -e
mkdir -p gpurun_out
for s in ${SHAPES:-3 4}; do
KMAN_RG_PASS=$s timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py -x -q --timeout 300 --timeout-method thread > gpurun_out/shape_tests.log 2>&1 || { tail -40 gpurun_out/shape_tests.log; exit 1; }
echo "shape $s: $(tail -1 gpurun_out/shape_tests.log)"
done
timeout -k 10 300 python -u tools/regionbench.py uniq ${BENCH:-KMAN_RG_PASS=0:0,KMAN_RG_PASS=3:0,KMAN_RG_PASS=4:0,KMAN_RG_PASS=0:0,KMAN_RG_PASS=3:0,KMAN_RG_PASS=4:0} 2>&1 | tee gpurun_out/shape.log
