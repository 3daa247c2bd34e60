# rg_pass without its end-of-tile barrier (base) vs with it (b7); region/parity/dist tests on base first
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04aa.log 2>&1 || { tail -40 gpurun_out/pytest_r04aa.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04aa.log
bash tools/ab/gpu_libab.sh r04aa 4 base b7
