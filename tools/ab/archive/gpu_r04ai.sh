# rg_finish: sizes and items of the block-id region loaded before the ticket returns (base) vs after (nospec); tests on base first
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04ai.log 2>&1 || { tail -40 gpurun_out/pytest_r04ai.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04ai.log
bash tools/ab/gpu_libab.sh r04ai 3 base nospec
BENCH_ARGS="--mode count" bash tools/ab/gpu_libab.sh r04aic 2 base nospec
