# rg_finish: wave priority 2 while a region's loads and row stores issue, 0 while it sorts (base) vs none (prio0)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04am.log 2>&1 || { tail -40 gpurun_out/pytest_r04am.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04am.log
bash tools/ab/gpu_libab.sh r04am 3 base prio0
BENCH_ARGS="--mode count" bash tools/ab/gpu_libab.sh r04amc 2 base prio0
