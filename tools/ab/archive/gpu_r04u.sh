# finish: clear / scan only the counter words a pass uses (base) vs all 256 (nw0); region tests on base first
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04u.log 2>&1 || { tail -40 gpurun_out/pytest_r04u.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04u.log
bash tools/ab/gpu_libab.sh r04u 3 base nw0
