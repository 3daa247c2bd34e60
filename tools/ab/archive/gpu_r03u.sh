# dist tests + config-4 line (statistical capacities, makespan H); rg_pass early prefetch (shape 8) A/B + its parity
set -e
mkdir -p gpurun_out
T="timeout -k 10"
$T 500 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_config3.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/u_tests.log 2>&1 || { tail -30 gpurun_out/u_tests.log; exit 1; }
tail -1 gpurun_out/u_tests.log
bash tools/gpu_cfg4ab.sh u KMAN_DROUND_PAD "1"
KMAN_RG_PASS=8 $T 500 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/u_tests8.log 2>&1 || { tail -30 gpurun_out/u_tests8.log; exit 1; }
tail -1 gpurun_out/u_tests8.log
bash tools/gpu_ab.sh u KMAN_RG_PASS "5 8" 2
