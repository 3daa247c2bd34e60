# rg_extract store loop: per-digit output base + item bound precomputed (base) vs the r04s tree (old); region + dist GPU tests on base first
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py tests/test_gpu_canonical.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04t.log 2>&1 || { tail -40 gpurun_out/pytest_r04t.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04t.log
bash tools/ab/gpu_libab.sh r04t 3 base old
