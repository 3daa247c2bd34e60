# rg_extract tile size with atomic cursors: EI 8 (4 blocks/CU) / 12 / 16 A/B + parity at 8
set -e
mkdir -p gpurun_out
KMAN_RG_EI=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_region.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/w_tests.log 2>&1 || { tail -30 gpurun_out/w_tests.log; exit 1; }
tail -1 gpurun_out/w_tests.log
bash tools/gpu_ab.sh w KMAN_RG_EI "12 8 16" 2
