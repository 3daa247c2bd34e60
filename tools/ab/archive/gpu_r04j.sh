# line-interleaved pass-1 layout (RG_ILV): region tests on the default build, then A/B vs the contiguous layout
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_canonical.py tests/test_gpu_config3.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04j.log 2>&1 || { tail -40 gpurun_out/pytest_r04j.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04j.log
bash tools/ab/gpu_libab.sh r04j 3 base noilv
