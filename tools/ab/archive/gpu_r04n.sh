# LDS round trips issued back to back (RG_PIPE): region/parity/canonical/config3/dist GPU tests on the default build, then A/B vs RG_PIPE=0
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_canonical.py tests/test_gpu_config3.py tests/test_gpu_dist_region.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04n.log 2>&1 || { tail -40 gpurun_out/pytest_r04n.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04n.log
bash tools/ab/gpu_libab.sh r04n 3 base nopipe
